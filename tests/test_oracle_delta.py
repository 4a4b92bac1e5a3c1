"""The what-if delta digest (test infrastructure, CPU only).

oracle_whatif_delta_digest hashes each unit's changed nodes with their new distance and
next-hop bytes in C; oracle.delta_digest computes the same from a CSR delta such as
openr_spf_whatif_delta returns. Here both sides come from the oracle: the CSR is built
from explicit runSpf(src) / runSpf(src, {link}) rows (LinkState.cpp:808-882), so the GPU
tests can compare a device delta with the C digest at full size.
"""
import numpy as np

from openr_amd import topology as T
from oracle import Oracle, delta_digest


def explicit_delta(o, g, links, sources, nb, use_metric=True):
    base = {int(s): o.run_spf(int(s), use_metric) for s in sources}
    ptr, node, dist, nh, counts = [0], [], [], [], []
    for l in links:
        for s in sources:
            r = o.run_spf(int(s), use_metric, [int(l)])
            b = base[int(s)]
            ch = np.nonzero((r.dist != b.dist) | np.any(r.nh != b.nh, axis=1))[0]
            node.extend(ch.tolist())
            dist.extend(r.dist[ch].tolist())
            rows = np.zeros((len(ch), nb), dtype=np.uint8)
            rows[:, : r.nh.shape[1]] = r.nh[ch, :nb]
            nh.append(rows)
            ptr.append(ptr[-1] + len(ch))
            counts.append(len(ch))
    return (np.array(ptr, dtype=np.uint64), np.array(node, dtype=np.uint32), np.array(dist, dtype=np.uint64),
            np.concatenate(nh) if nh else np.zeros((0, nb), np.uint8), np.array(counts, dtype=np.uint32))


def test_delta_digest_matches_explicit_rows():
    g = T.wan(120, 300, 64, seed=3)
    o = Oracle(g)
    links = list(range(0, g.num_links, 7))
    sources = [0, 17, 63, 119]
    for nb in (o.nh_bytes, o.nh_bytes + 3):  # the caller may ask for wider next-hop entries
        ptr, node, dist, nh, counts = explicit_delta(o, g, links, sources, nb)
        changed, dig = o.whatif_delta_digest(links, sources, nb)
        np.testing.assert_array_equal(changed.ravel(), counts)
        np.testing.assert_array_equal(dig.ravel(), delta_digest(ptr, node, dist, nh))
        assert counts.sum() > 0
    # a perturbed entry changes its unit's digest
    u = int(np.nonzero(counts)[0][0])
    dist2 = dist.copy()
    dist2[int(ptr[u])] += np.uint64(1)
    d2 = delta_digest(ptr, node, dist2, nh)
    assert d2[u] != dig.ravel()[u]
