"""Philox4x32-10 oracle against the Random123 known-answer vectors (kat_vectors)."""
import numpy as np

from oracle.philox import STREAM_DEMAND, draw_words, philox4x32_10, seed_key

KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def test_known_answers():
    for ctr, key, want in KAT:
        got = philox4x32_10(np.array(ctr, dtype=np.uint32), np.array(key, dtype=np.uint32))
        assert [int(x) for x in got] == list(want)


def test_vectorised_matches_scalar():
    rng = np.random.RandomState(0)
    ctr = rng.randint(0, 2 ** 32, size=(50, 4), dtype=np.uint64).astype(np.uint32)
    key = rng.randint(0, 2 ** 32, size=2, dtype=np.uint64).astype(np.uint32)
    batch = philox4x32_10(ctr, key)
    for i in range(50):
        assert np.array_equal(batch[i], philox4x32_10(ctr[i], key))


def test_word_layout():
    seed = 0x1234_5678_9ABC_DEF0
    w = draw_words(seed, [3, 7], episode=5, n_words=9, stream=STREAM_DEMAND)
    assert w.shape == (2, 9)
    blk = philox4x32_10(np.array([7, 5, 2, STREAM_DEMAND], dtype=np.uint32), seed_key(seed))
    assert w[1, 8] == blk[0]
    blk = philox4x32_10(np.array([3, 5, 1, STREAM_DEMAND], dtype=np.uint32), seed_key(seed))
    assert list(w[0, 4:8]) == list(blk)
