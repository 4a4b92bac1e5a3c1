"""Loaders for tests/golden/*.json (reference test expectations)."""
import json
import os

from openr_amd import topology as T

HERE = os.path.dirname(os.path.abspath(__file__))


def load(name="reference_spf_cases.json"):
    with open(os.path.join(HERE, "golden", name)) as f:
        return json.load(f)


def build(case):
    """CSR mirror of a golden case (adj_map -> getLinkState fixture; dbs -> explicit adjacencies)."""
    if "adj_map" in case:
        adj_map = {int(k): [tuple(x) if isinstance(x, list) else x for x in v] for k, v in case["adj_map"].items()}
        return T.from_adj_map(adj_map)
    dbs = []
    for db in case["dbs"]:
        adjs = [T.Adjacency(a[0], a[1], a[2], a[3]) for a in db["adjs"]]
        dbs.append(T.AdjacencyDatabase(db["node"], adjs, db.get("overloaded", False)))
    return T.build_csr(dbs)


def spf_cases():
    return [c for c in load()["cases"] if "spf" in c]


def kth_cases():
    return [c for c in load()["cases"] if "kth" in c]


def hop_cases():
    return [c for c in load()["cases"] if "hops" in c]
