"""Oracle RNG pinned by known-answer vectors (Random123 kat_vectors, philox4x32 R=10)."""
import numpy as np

from oracle.philox import estimator_permutation, philox4x32_10, splitmix64_next, uniforms


def test_philox_kat():
    kat = [
        ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
        ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
        ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
         (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
    ]
    for ctr, key, want in kat:
        got = philox4x32_10(*ctr, *key)
        assert tuple(int(v) for v in got) == want


def test_splitmix64_kat():
    # reference outputs of splitmix64 seeded with 0 (Vigna's splitmix64.c)
    s = 0
    outs = []
    for _ in range(3):
        s, o = splitmix64_next(s)
        outs.append(o)
    assert outs == [0xE220A8397B1DCDAF, 0x6E789E6AA1B965F4, 0x06C45D188009454F]


def test_uniforms_range_and_independence():
    u = uniforms(123, 7, 100_000)
    assert u.dtype == np.float32 and u.min() >= 0.0 and u.max() < 1.0
    assert abs(u.mean() - 0.5) < 0.005 and abs(u.std() - np.sqrt(1 / 12)) < 0.005
    v = uniforms(123, 8, 100_000)
    assert abs(np.corrcoef(u, v)[0, 1]) < 0.02
    # row offset addressing is consistent
    np.testing.assert_array_equal(uniforms(123, 7, 10, row_offset=5), u[5:15])


def test_permutation_is_a_permutation():
    for F in (1, 2, 7, 19):
        for e in range(8):
            p = estimator_permutation(0, e, F)
            assert sorted(p.tolist()) == list(range(F))
