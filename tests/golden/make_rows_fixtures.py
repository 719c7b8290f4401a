"""Writes tests/golden/rows_exceptional.json: chosen-scalar signatures under
the key Q = G whose partial sums meet inside the latency path's row tree
(tests/rowtree.py), for the three row geometries the parity tests serve --
(29, 21) (100 keys, six waves), (29, 24) (4 keys, six waves) and (29, 20)
(seven waves).  Expected bits come from the oracle restatement
(oracle/p256.py) and are re-checked against the C oracle by
tests/test_rowtree.py.  Test infrastructure only; run from the repo root:

    python tests/golden/make_rows_fixtures.py
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import rowtree  # noqa: E402

GEOMETRIES = [(29, 21), (29, 24), (29, 20)]


def main():
    out = {"note": "tests/rowtree.py vectors(gq, seed=1): key 0 = G; u1/u2 are the scalars the verifier "
                   "recomputes, events the row-tree meetings (tree_events), exceptional = the row kernel "
                   "must take its exact path, expect = oracle/p256.py verify",
           "geometries": {}}
    for gq in GEOMETRIES:
        vs = rowtree.vectors(gq, seed=1)
        out["geometries"][f"{gq[0]},{gq[1]}"] = [
            {"kind": v["kind"], "hash": v["hash"].hex(), "r": f"{v['r']:064x}", "s": f"{v['s']:064x}",
             "u1": f"{v['u1']:064x}", "u2": f"{v['u2']:064x}", "events": [list(e) for e in v["events"]],
             "exceptional": v["exceptional"], "expect": bool(v["expect"])} for v in vs]
        print(gq, len(vs), "vectors,", sum(v["expect"] for v in vs), "valid", file=sys.stderr)
    with open(os.path.join(HERE, "rows_exceptional.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
