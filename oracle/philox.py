"""Philox4x32-10 counter-based RNG, NumPy restatement — TEST INFRASTRUCTURE ONLY.

The reference (gym_supplychain) has no RNG in BeerGameEnv (beergame_env.py:6-181 has no
seed/RandomState); the Poisson demand of BASELINE config 2 is a builder-supplied input
(SURVEY.md F2). The device draws it with Philox4x32-10 (Salmon et al., SC'11,
"Parallel random numbers: as easy as 1, 2, 3"; algorithm as published in Random123).
This file restates that published algorithm independently of the HIP header so the
two can be checked against each other and against the Random123 known-answer vectors
(tests/test_oracle_philox.py).

Counter layout used by scgpu (see DESIGN.md "Randomness"):
    key = (seed & 0xffffffff, seed >> 32)
    ctr = (global_env_id, episode, word_block, stream)
one call yields four uint32 words.
"""
import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)

STREAM_DEMAND = 0
STREAM_ACTION = 1


def philox4x32_10(ctr, key):
    """Vectorised Philox4x32-10.

    ctr: uint32 array [..., 4]; key: uint32 array [..., 2] (broadcastable).
    Returns uint32 array [..., 4].
    """
    ctr = np.asarray(ctr, dtype=np.uint32)
    key = np.asarray(key, dtype=np.uint32)
    c0, c1, c2, c3 = (ctr[..., i].astype(np.uint32) for i in range(4))
    k0 = np.broadcast_to(key[..., 0], c0.shape).astype(np.uint32)
    k1 = np.broadcast_to(key[..., 1], c0.shape).astype(np.uint32)
    for r in range(10):
        p0 = c0.astype(np.uint64) * M0
        p1 = c2.astype(np.uint64) * M1
        hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
        lo0 = (p0 & MASK32).astype(np.uint32)
        hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
        lo1 = (p1 & MASK32).astype(np.uint32)
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        if r < 9:
            k0 = ((k0.astype(np.uint64) + np.uint64(W0)) & MASK32).astype(np.uint32)
            k1 = ((k1.astype(np.uint64) + np.uint64(W1)) & MASK32).astype(np.uint32)
    return np.stack([c0, c1, c2, c3], axis=-1)


def seed_key(seed):
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    return np.array([seed & 0xFFFFFFFF, seed >> 32], dtype=np.uint32)


def draw_words(seed, env_ids, episode, n_words, stream):
    """uint32 words [len(env_ids), n_words]: word j of env e comes from
    philox(ctr=(e, episode, j // 4, stream))[j % 4]."""
    env_ids = np.asarray(env_ids, dtype=np.uint64)
    n_blocks = (n_words + 3) // 4
    ctr = np.zeros((len(env_ids), n_blocks, 4), dtype=np.uint32)
    ctr[..., 0] = (env_ids & MASK32).astype(np.uint32)[:, None]
    ctr[..., 1] = np.uint32(episode & 0xFFFFFFFF)
    ctr[..., 2] = np.arange(n_blocks, dtype=np.uint32)[None, :]
    ctr[..., 3] = np.uint32(stream)
    out = philox4x32_10(ctr, seed_key(seed))
    return out.reshape(len(env_ids), n_blocks * 4)[:, :n_words]
