"""The warm-start cache across the carried point counts (Own.wsm, cp_physics.h ws_count).

Each lane loads its island's warm-start id words once per launch, keeps their point counts in 3 bits per pair,
and a pair the broadphase separates neither reads its cache entry nor compares the id word: it is rewritten when
its old count was > 0 or the word was not a prefix (ids, then 0xFF padding).  The oracle rewrites every slot of
every pair every substep, so any difference in that decision shows in the state.  Seeded through cp_set_state:
prefix words with 1-4 ids and matching impulses, words that are not prefixes (0xFF in front of an id byte,
random words) with random impulses, on pairs that are in contact and pairs that are far apart; then steps with
autoreset on every kernel-shape pair (fp32), obs and the whole state SoA bit for bit.
(Excluded by construction: an all-0xFF word over non-zero impulses, which no kernel or cp_init writes; the
kernels assume those impulses are 0, as before round 5.)"""
import numpy as np
import pytest
import torch

from cartpoleplusplus_amd import abi, native
from cartpoleplusplus_amd.batched import BatchedCartpole
from tests.test_gpu_parity import SHAPES, SHAPE_IDS, _assert_same, _np

pytestmark = pytest.mark.gpu

B, STEPS = 96, 12


def _seed_cache(st, rng):
    ids = st.view(np.uint32)
    for e in range(B):
        for p in range(2):
            for j in range(abi.CP_ISLAND_PAIRS):
                kind = (e * 7 + p * 3 + j) % 5
                if kind == 0:      # a prefix of n ids (the kernels' own words)
                    n = int(rng.integers(1, 5))
                    b = list(rng.integers(0, 200, n)) + [0xFF] * (4 - n)
                    lam = [float(rng.uniform(0, 2)) if k < n else 0.0 for k in range(4)]
                elif kind == 1:    # not a prefix: 0xFF before an id byte
                    b = [0xFF, int(rng.integers(0, 200)), 0xFF, int(rng.integers(0, 200))]
                    lam = list(rng.uniform(0, 2, 4))
                elif kind == 2:    # a random word
                    b = list(rng.integers(0, 256, 4))
                    lam = list(rng.uniform(-1, 2, 4))
                else:              # the empty word (impulses 0: the invariant)
                    b = [0xFF] * 4
                    lam = [0.0] * 4
                ids[abi.CP_SF_WS_ID(p, j), e] = np.uint32(b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24))
                for k in range(4):
                    st[abi.CP_SF_WS_LAM(p, j, k), e] = lam[k]
    return st


def _run(O, shape):
    cfg = native.default_config(num_envs=B, action_repeats=3, initial_force=55.0, seed=29, autoreset=1,
                                max_episode_len=8)
    gpu = BatchedCartpole(B, 0, config=abi.cp_config.from_buffer_copy(cfg))
    gpu.set_kernel_shape(*shape)
    orc = O.Envs(abi.cp_config.from_buffer_copy(cfg))
    _assert_same(_np(gpu.reset()), orc.reset(), "reset obs")
    rng = np.random.default_rng(31)
    for t in range(3):   # into the episode: some pairs in contact, the cross pairs far apart
        a = rng.integers(0, 5, (B, 2)).astype(np.int8)
        gpu.step(torch.from_numpy(a).cuda())
        orc.step(a)
    st = _seed_cache(_np(gpu.get_state()).copy(), np.random.default_rng(37))
    gpu.set_state(torch.from_numpy(st).cuda())
    orc.set_state(np.ascontiguousarray(st))
    for t in range(STEPS):
        a = rng.integers(0, 5, (B, 2)).astype(np.int8)
        go, _, gd = gpu.step(torch.from_numpy(a).cuda())
        oo, _, od = orc.step(a)
        _assert_same(_np(go), oo, f"obs step {t}")
        _assert_same(_np(gd), od, f"done step {t}")
    g, o = _np(gpu.get_state()), orc.get_state()
    assert np.array_equal(g.view(np.uint32), o.view(np.uint32)), "state bits"
    gpu.close()


@pytest.mark.parametrize("shape", SHAPES, ids=SHAPE_IDS)
def test_wscache_seeded_words_vs_oracle(oracle_mod, shape):
    _run(oracle_mod, shape)
