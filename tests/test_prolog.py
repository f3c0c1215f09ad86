"""TCAP <-> Prolog bridge (reference src/optimizerBenchmark: prologGenerator.cc / prologToTCAP.pl) and the
movie-star benchmark graph it was written for."""
from netsdb_amd import _ext
from netsdb_amd.client import PDBClient
from netsdb_amd.examples import movies
from netsdb_amd.logical_plan.prolog import parse_fact, prolog_to_tcap, tcap_to_prolog
from netsdb_amd.logical_plan.tcap import compile_tcap


def _canon(tcap: str):
    return sorted(str(sorted(a.items())) for a in
                  ({k: v for k, v in a.items() if k != "line"} for a in _ext.native().parse_tcap(tcap)))


def test_movie_tcap_prolog_roundtrip():
    tcap = compile_tcap([movies.plan()]).tcap
    rules = tcap_to_prolog(tcap)
    kinds = {parse_fact(r)[0] for r in rules}
    assert {"node", "link", "scan", "apply", "filter", "hashleft", "hashright", "join", "output"} <= kinds
    # every atom has exactly one node fact; scans hang off the virtual root
    atoms = _ext.native().parse_tcap(tcap)
    assert sum(r.startswith("node(") for r in rules) == len(atoms)
    assert sum(r.startswith("link(virtualRootNode") for r in rules) == 2
    back = prolog_to_tcap(rules)
    assert _canon(back) == _canon(tcap)
    # shuffled facts still rebuild a valid, producer-before-consumer TCAP
    import random

    shuffled = list(rules)
    random.Random(1).shuffle(shuffled)
    again = prolog_to_tcap(shuffled)
    assert _canon(again) == _canon(tcap)
    seen = set()
    for a in _ext.native().parse_tcap(again):
        for k in ("input", "input2"):
            if a[k]["name"]:
                assert a[k]["name"] in seen
        seen.add(a["output"]["name"])


def test_parse_fact_quoting():
    name, args = parse_fact("apply('x_1', in, 'Proj', '==_2').")
    assert name == "apply" and args == ["x_1", "in", "Proj", "==_2"]
    name, args = parse_fact("link(a, b, ['A', b_c], [], [x]).")
    assert args[2] == ["A", "b_c"] and args[3] == [] and args[4] == ["x"]


def test_movie_join_runs(tmp_path):
    c = PDBClient(root=str(tmp_path), page_size=1 << 12)
    stars, roles = movies.generate()
    stars[0].birthYear = 1960
    roles.append(movies.StarsIn("m", stars[0].name, 1990))
    got = sorted(o.name for o in movies.run(c, stars, roles))
    assert got == movies.reference(stars, roles) and got
