"""TCAP <-> Prolog rules — the optimizer-benchmark bridge.

Reference: src/optimizerBenchmark/source/prologGenerator.cc (``parseTCAPtoProlog``: one ``node``
fact per atomic computation, one ``link`` fact per input edge with the output / input /
projection attribute lists, one operator fact per atom) and prologToTCAP.pl (``tcapGenerator``:
rebuild TCAP text from those facts; the original line order is not kept).

Differences by design: names are emitted as quoted Prolog atoms (``'SelectionComp_1'``) instead of
lower-casing their first letter, so the conversion is lossless and ``prolog_to_tcap`` rebuilds the
exact atoms; the inverse is implemented here (a small fact reader + topological ordering) rather
than in a Prolog interpreter, which this image does not ship.  The TCAP text is parsed by the
native parser (``_ext.native().parse_tcap``) — the same front end the planner uses.

Fact vocabulary::

    node(Out, Type, Comp).                          Type in scan apply filter hashleft hashright
                                                    hashone flatten join aggregate partition output
    link(Out, In, [OutAtts], [InAtts], [ProjAtts]). one per input edge; a scan links from
                                                    virtualRootNode with empty lists
    scan(Out, Db, Set).          apply(Out, In, Proj, Lambda).   filter(Out, In, Proj).
    hashleft(Out, In, Proj, Lambda).  hashright(Out, In, Proj, Lambda).  hashone(Out, In, Proj).
    flatten(Out, In, Proj).      join(Out, In, Proj, RIn, RProj).   aggregate(Out, In).
    partition(Out, In).          output(Out, In, Db, Set).
"""
from __future__ import annotations

import re
from typing import Dict, List, Sequence, Tuple

ROOT = "virtualRootNode"
_PLAIN = re.compile(r"^[a-z][A-Za-z0-9_]*$")


def _atom(s: str) -> str:
    s = str(s)
    if _PLAIN.match(s) and s != ROOT:
        return s
    return "'" + s.replace("\\", "\\\\").replace("'", "\\'") + "'"


def _list(xs: Sequence[str]) -> str:
    return "[" + ", ".join(_atom(x) for x in xs) + "]"


def _atoms_of(tcap_or_atoms) -> List[dict]:
    if isinstance(tcap_or_atoms, str):
        from .. import _ext

        return list(_ext.native().parse_tcap(tcap_or_atoms))
    return list(tcap_or_atoms)


def tcap_to_prolog(tcap_or_atoms) -> List[str]:
    """One fact per line: node + link(s) + the operator fact of every atomic computation."""
    rules: List[str] = []
    for a in _atoms_of(tcap_or_atoms):
        t = a["type"].lower()
        out, o_atts = a["output"]["name"], a["output"]["atts"]
        rules.append(f"node({_atom(out)}, {t}, {_atom(a['comp'])}).")
        if t == "scan":
            rules.append(f"link({ROOT}, {_atom(out)}, {_list(o_atts)}, [], []).")
        else:
            rules.append(f"link({_atom(out)}, {_atom(a['input']['name'])}, {_list(o_atts)}, "
                         f"{_list(a['input']['atts'])}, {_list(a['projection']['atts'])}).")
            if t == "join":
                rules.append(f"link({_atom(out)}, {_atom(a['input2']['name'])}, {_list(o_atts)}, "
                             f"{_list(a['input2']['atts'])}, {_list(a['projection2']['atts'])}).")
        i, p = _atom(a["input"]["name"]), _atom(a["projection"]["name"])
        if t == "scan":
            rules.append(f"scan({_atom(out)}, {_atom(a['db'])}, {_atom(a['set'])}).")
        elif t in ("apply", "hashleft", "hashright"):
            rules.append(f"{t}({_atom(out)}, {i}, {p}, {_atom(a['lambda'])}).")
        elif t in ("filter", "hashone", "flatten"):
            rules.append(f"{t}({_atom(out)}, {i}, {p}).")
        elif t == "join":
            rules.append(f"join({_atom(out)}, {i}, {p}, {_atom(a['input2']['name'])}, "
                         f"{_atom(a['projection2']['name'])}).")
        elif t in ("aggregate", "partition"):
            rules.append(f"{t}({_atom(out)}, {i}).")
        elif t == "output":
            rules.append(f"output({_atom(out)}, {i}, {_atom(a['db'])}, {_atom(a['set'])}).")
        else:
            raise ValueError(f"{a['type']} is not supported by the Prolog bridge")
    return rules


# ------------------------------------------------------------------ fact reader
_TOK = re.compile(r"\s*(?:(?P<q>'(?:\\.|[^'\\])*')|(?P<w>[A-Za-z0-9_=<>!+\-*/.]+)|(?P<p>[()\[\],]))")


def _tokens(s: str):
    pos = 0
    while pos < len(s):
        m = _TOK.match(s, pos)
        if not m or m.end() == pos:
            if s[pos:].strip() == "":
                return
            raise ValueError(f"bad Prolog text at {s[pos:pos + 20]!r}")
        pos = m.end()
        if m.group("q"):
            yield ("a", re.sub(r"\\(.)", r"\1", m.group("q")[1:-1]))
        elif m.group("w"):
            yield ("a", m.group("w"))
        else:
            yield ("p", m.group("p"))


def parse_fact(line: str) -> Tuple[str, list]:
    """``name(arg, [a, b], ...).`` -> (name, [str | list[str]])."""
    line = line.strip()
    if line.endswith("."):
        line = line[:-1]
    toks = list(_tokens(line))
    if len(toks) < 3 or toks[0][0] != "a" or toks[1] != ("p", "("):
        raise ValueError(f"not a fact: {line!r}")
    args: list = []
    k = 2
    while k < len(toks):
        kind, v = toks[k]
        if (kind, v) == ("p", ")"):
            break
        if (kind, v) == ("p", ","):
            k += 1
            continue
        if (kind, v) == ("p", "["):
            lst = []
            k += 1
            while toks[k] != ("p", "]"):
                if toks[k][0] == "a":
                    lst.append(toks[k][1])
                k += 1
            args.append(lst)
        else:
            args.append(v)
        k += 1
    return toks[0][1], args


def prolog_to_tcap(rules: Sequence[str]) -> str:
    """Rebuild TCAP text from node/link/operator facts (prologToTCAP.pl ``tcapGenerator``): atoms are
    emitted in a topological order of the link graph (producers before consumers)."""
    facts: List[Tuple[str, list]] = []
    for r in rules:
        for piece in str(r).splitlines():
            if piece.strip() and not piece.strip().startswith("%"):
                facts.append(parse_fact(piece))
    nodes: Dict[str, Tuple[str, str]] = {}
    links: Dict[str, List[list]] = {}
    ops: Dict[str, Tuple[str, list]] = {}
    order: List[str] = []
    for name, args in facts:
        if name == "node":
            nodes[args[0]] = (args[1], args[2])
            order.append(args[0])
        elif name == "link":
            links.setdefault(args[0] if args[0] != ROOT else args[1], []).append(args)
        else:
            ops[args[0]] = (name, args)

    def spec(n: str, atts: Sequence[str]) -> str:
        return f"{n}({', '.join(atts)})"

    def q(s: str) -> str:
        return "'" + s + "'"

    emitted: Dict[str, str] = {}
    deps = {o: [ln[1] for ln in links.get(o, []) if ln[0] != ROOT] for o in order}
    seen, topo = set(), []

    def visit(o):
        if o in seen:
            return
        seen.add(o)
        for d in deps.get(o, []):
            if d in nodes:
                visit(d)
        topo.append(o)

    for o in order:
        visit(o)
    for o in topo:
        typ, comp = nodes[o]
        op, args = ops[o]
        ls = links.get(o, [])
        out_atts = ls[0][2] if ls else []
        if typ == "scan":
            line = f"{spec(o, out_atts)} <= SCAN ({q(args[1])}, {q(args[2])}, {q(comp)})"
        else:
            l0 = ls[0]
            inp, proj = spec(l0[1], l0[3]), spec(l0[1], l0[4])
            if typ in ("apply", "hashleft", "hashright"):
                line = f"{spec(o, out_atts)} <= {typ.upper()} ({inp}, {proj}, {q(comp)}, {q(args[3])})"
            elif typ in ("filter", "hashone", "flatten"):
                line = f"{spec(o, out_atts)} <= {typ.upper()} ({inp}, {proj}, {q(comp)})"
            elif typ == "join":
                l1 = ls[1]
                line = (f"{spec(o, out_atts)} <= JOIN ({inp}, {proj}, {spec(l1[1], l1[3])}, "
                        f"{spec(l1[1], l1[4])}, {q(comp)})")
            elif typ in ("aggregate", "partition"):
                line = f"{spec(o, out_atts)} <= {typ.upper()} ({inp}, {q(comp)})"
            elif typ == "output":
                line = f"{spec(o, out_atts)} <= OUTPUT ({inp}, {q(args[2])}, {q(args[3])}, {q(comp)})"
            else:
                raise ValueError(f"unknown node type {typ}")
        emitted[o] = line
    return "\n".join(emitted[o] for o in topo) + "\n"


__all__ = ["tcap_to_prolog", "prolog_to_tcap", "parse_fact", "ROOT"]
