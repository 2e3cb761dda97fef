"""The CPU restatement (oracle/) against the reference's golden vectors and
against NumPy / CPython primitives.  No GPU."""
import random

import numpy as np
import pytest

from golden_util import case_names, dff_hash, load_case
from oracle import oracle as O

CASES = case_names()


def test_cases_present():
    assert {"neumann_12x12_N8", "neumann_12x12_N32", "moore_12x12_N32",
            "main_50x50_N100", "neumann_64x64_N512"} <= set(CASES)


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference_goldens(name):
    case = load_case(name)
    core = O.Core(case.map, case.sff, case.params)
    for ep in case.episodes:
        np_rng, py_rng = O.seeded_np(ep.seed), O.seeded_py(ep.seed)
        pos = core.init_agents_mt(case.N, np_rng)
        assert np.array_equal(pos, ep.init), f"seed {ep.seed}: initial placement"
        dff = np.zeros(case.map.shape, dtype=np.float32)
        for t in range(len(ep.counts)):
            pos = core.step_mt(pos, dff, np_rng, py_rng)
            assert np.array_equal(pos, ep.cells[t]), f"seed {ep.seed} step {t}: positions"
            assert dff_hash(dff) == int(ep.hashes[t]), f"seed {ep.seed} step {t}: DFF bits"
            if ep.full:
                assert np.array_equal(dff.view(np.uint32), ep.full[t].view(np.uint32))
        assert [O.lib().ffo_mt_next(np_rng) for _ in range(4)] == list(ep.np_tail), "np stream"
        assert [O.lib().ffo_mt_next(py_rng) for _ in range(4)] == list(ep.py_tail), "py stream"


def test_mt_streams_match_interpreter():
    m = O.seeded_np(42)
    assert O.lib().ffo_mt_next(m) == 1608637542
    rs = np.random.RandomState(42)
    m = O.MT.from_numpy(rs)
    assert [O.lib().ffo_mt_u53(m) for _ in range(8)] == list(rs.random_sample(8))
    p = np.zeros(100, dtype=np.int64)
    rs = np.random.RandomState(42)
    O.lib().ffo_np_permutation(O.MT.from_numpy(rs), 100, O._ptr(p))
    assert list(p[:8]) == [83, 53, 70, 45, 44, 39, 22, 80]
    r = random.Random(42)
    m = O.seeded_py(42)
    assert O.lib().ffo_mt_u53(m) == r.random() == 0.6394267984578837
    m = O.MT.from_python(r)
    for n in (2, 3, 5, 7, 8, 9, 100, 65535):
        assert [O.lib().ffo_py_randbelow(m, n) for _ in range(20)] == [r._randbelow(n) for _ in range(20)]


def test_mt_state_roundtrip_with_interpreter():
    rs = np.random.RandomState(7)
    rs.random_sample(1000)
    m = O.MT.from_numpy(rs)
    O.lib().ffo_mt_u53(m)
    m.to_numpy(rs)
    ref = np.random.RandomState(7)
    ref.random_sample(1001)
    assert rs.random_sample() == ref.random_sample()
    r = random.Random(9)
    m = O.MT.from_python(r)
    O.lib().ffo_mt_next(m)
    m.to_python(r)
    r2 = random.Random(9)
    r2.getrandbits(32)
    assert r.random() == r2.random()


def test_np_exp_float32_sampled():
    rs = np.random.RandomState(1)
    x = rs.uniform(-104, 0, 4_000_000).astype(np.float32)
    x = np.concatenate([x, np.float32([0.0, -0.0, -np.inf, -103.9720, -103.97209, -87.3, -1e-30]),
                        -np.abs(rs.standard_normal(1_000_000).astype(np.float32))])
    assert np.array_equal(O.np_expf(x).view(np.uint32), np.exp(x).view(np.uint32))


@pytest.mark.slow
def test_np_exp_float32_exhaustive_negative():
    """Every float32 in [-104, -0] (≈1.12e9 values), in chunks."""
    lo = np.float32(-0.0).view(np.uint32)
    hi = np.float32(-104.0).view(np.uint32)
    chunk = 1 << 26
    for start in range(int(lo), int(hi) + 1, chunk):
        bits = np.arange(start, min(start + chunk, int(hi) + 1), dtype=np.uint32)
        x = bits.view(np.float32)
        assert np.array_equal(O.np_expf(x).view(np.uint32), np.exp(x).view(np.uint32)), hex(start)


def test_np_sum_order():
    rs = np.random.RandomState(3)
    for n in range(1, 18):
        for _ in range(2000):
            v = (rs.uniform(0, 1, n) * 10.0 ** rs.uniform(-8, 0, n)).astype(np.float32)
            assert O.np_sumf(v).view(np.uint32) == np.float32(v.sum()).view(np.uint32), n


def test_update_dff_matches_numpy_expression():
    """update_dff restated vs the reference's own NumPy expression (model/ffm_core.py:106-117)."""
    rs = np.random.RandomState(5)
    for nbname in ("neumann", "moore"):
        core = O.Core(np.zeros((9, 13), np.uint8), np.zeros((9, 13), np.float32),
                      {"diffuse": 0.3, "decay": 0.15, "neighborhood": nbname})
        nbs = [(-1, 0), (1, 0), (0, -1), (0, 1)] if nbname == "neumann" else \
            [(-1, -1), (-1, 0), (-1, 1), (0, -1), (0, 1), (1, -1), (1, 0), (1, 1)]
        d = (rs.exponential(1.0, (9, 13)) * (rs.uniform(size=(9, 13)) < 0.6)).astype(np.float32)
        new = (1 - 0.15) * (1 - 0.3) * d
        padded = np.pad(new, 1, mode="constant")
        for dx, dy in nbs:
            new += 0.15 * (1 - 0.3) / len(nbs) * padded[1 + dx:new.shape[0] + 1 + dx, 1 + dy:new.shape[1] + 1 + dy]
        new[new < 1e-4] = 0
        got = d.copy()
        core.update_dff(got)
        assert np.array_equal(got.view(np.uint32), new.view(np.uint32))


def test_philox_known_answer():
    # Random123 known-answer vectors for philox4x32-10.
    assert list(O.philox([0, 0, 0, 0], [0, 0])) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert list(O.philox([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2)) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert list(O.philox([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0])) == \
        [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_philox_batch_invariants():
    """Philox mode: env results independent of batch slicing and thread count."""
    from ffm_amd.data import make_room, l1_sff
    m = make_room(12, 12)
    core = O.Core(m, l1_sff(m), {"neighborhood": "neumann"})
    E, A = 64, 32
    def run(nthreads, split):
        pos = np.zeros((E, A), np.uint16)
        cnt = np.zeros(E, np.int32)
        dff = np.zeros((E, 12, 12), np.float32)
        ep = np.zeros(E, np.int32)
        tot = 0
        for t in range(40):
            for lo, hi in split:
                tot += core.step_philox_batch(pos[lo:hi], cnt[lo:hi], dff[lo:hi], ep[lo:hi], 42, t,
                                              True, 32, env_base=lo, nthreads=nthreads)
        return pos, cnt, dff, ep, tot
    a = run(1, [(0, E)])
    b = run(4, [(0, 17), (17, 40), (40, E)])
    for x, y in zip(a[:4], b[:4]):
        assert np.array_equal(x, y)
    assert a[4] == b[4] and a[4] > 0
    assert (a[3] >= 1).all()
    # positions of live agents are distinct free/exit-free cells
    for e in range(E):
        c = a[0][e, :a[1][e]]
        assert len(set(c.tolist())) == len(c)
        assert (m.reshape(-1)[c] == 0).all()
