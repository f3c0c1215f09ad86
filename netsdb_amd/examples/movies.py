"""Movie-star optimizer benchmark (reference: src/optimizerBenchmark — MovieStar, StarsIn,
ScanMovieStarSet, ScanStarsInSet, SimpleMovieSelection (birthYear == checkBirthYear),
SimpleMovieJoin (MovieStar.name == StarsIn.starName, project the star), SimpleMovieWrite, and
tcapGenerator.cc which compiles that graph to TCAP and hands it to the Prolog rule generator).

``plan()`` builds the same computation graph; ``run()`` executes it through the engine; the TCAP /
Prolog round trip lives in :mod:`netsdb_amd.logical_plan.prolog`.
"""
from __future__ import annotations

from typing import List

from ..computations import JoinComp, ScanSet, SelectionComp, WriteSet
from ..lambdas import make_lambda, make_lambda_from_member
from ..objects import PDBObject


class MovieStar(PDBObject):
    name: str
    address: str
    gender: str
    birthYear: int
    checkBirthYear: int


class StarsIn(PDBObject):
    movieTitle: str
    starName: str
    movieYear: int


def movie_star(name: str, address: str, gender: str, birth_year: int) -> MovieStar:
    """MovieStar(name, address, gender, birthYear); checkBirthYear defaults to 1960 as in the reference."""
    return MovieStar(name, address, gender, birth_year, 1960)


class SimpleMovieSelection(SelectionComp):
    def get_selection(self, s):
        return make_lambda_from_member(s, "birthYear") == make_lambda_from_member(s, "checkBirthYear")

    def get_projection(self, s):
        return make_lambda(s, lambda r: r)


class SimpleMovieJoin(JoinComp):
    def get_selection(self, star, role):
        return make_lambda_from_member(star, "name") == make_lambda_from_member(role, "starName")

    def get_projection(self, star, role):
        return make_lambda(star, lambda r: r)


def plan(db: str = "movies", out: str = "stars1960"):
    """Scan stars -> select birthYear == 1960 -> join StarsIn on name -> write."""
    sel = SimpleMovieSelection().set_input(ScanSet(db, "stars", MovieStar))
    j = SimpleMovieJoin()
    j.set_input(0, sel)
    j.set_input(1, ScanSet(db, "starsIn", StarsIn))
    return WriteSet(db, out).set_input(j)


def generate(n_stars: int = 40, n_roles: int = 120, seed: int = 0):
    import random

    rnd = random.Random(seed)
    stars = [movie_star(f"star{i}", f"{i} Main St", "FM"[i % 2], 1950 + rnd.randrange(20)) for i in range(n_stars)]
    roles = [StarsIn(f"movie{rnd.randrange(30)}", f"star{rnd.randrange(n_stars)}", 1970 + rnd.randrange(40))
             for _ in range(n_roles)]
    return stars, roles


def run(client, stars: List[MovieStar], roles: List[StarsIn], db: str = "movies", out: str = "stars1960"):
    client.create_database(db)
    client.create_set(db, "stars", MovieStar)
    client.create_set(db, "starsIn", StarsIn)
    client.create_set(db, out, MovieStar)
    client.send_data(db, "stars", stars)
    client.send_data(db, "starsIn", roles)
    client.execute_computations(plan(db, out), job_name="movie_join")
    return [o for o in client.get_set_iterator(db, out)]


def reference(stars, roles) -> List[str]:
    """One output row per (1960-born star, role) match, as the join emits it."""
    born = {s.name for s in stars if s.birthYear == 1960}
    return sorted(r.starName for r in roles if r.starName in born)


__all__ = ["MovieStar", "StarsIn", "movie_star", "SimpleMovieSelection", "SimpleMovieJoin", "plan", "generate",
           "run", "reference"]
