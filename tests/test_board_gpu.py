"""Parity of the device board-step / legal-mask / D4 kernels (oth_*_gpu through the C ABI)
against the reference-generated golden corpus and the oracle (bit-exact)."""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("az_native")
from oracle import board as ob  # noqa: E402


def dev(a):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    return torch.from_numpy(a).cuda()


def host_u64(t):
    return t.cpu().numpy().view(np.uint64)


def step_gpu(own, opp, act):
    n = len(own)
    d_own, d_opp = dev(np.asarray(own, np.uint64)), dev(np.asarray(opp, np.uint64))
    d_act = dev(np.asarray(act, np.uint8))
    o, p, lg = (torch.empty(n, dtype=torch.int64, device="cuda") for _ in range(3))
    st = torch.empty(n, dtype=torch.int16, device="cuda")
    nat.check(nat.lib.oth_step_gpu(nat.ptr(d_own), nat.ptr(d_opp), nat.ptr(d_act), nat.ptr(o),
                                   nat.ptr(p), nat.ptr(lg), nat.ptr(st), n, nat.stream_ptr()),
              "oth_step_gpu")
    torch.cuda.synchronize()
    return host_u64(o), host_u64(p), host_u64(lg), st.cpu().numpy().view(np.uint16)


def legal_gpu(own, opp):
    n = len(own)
    out = torch.empty(n, dtype=torch.int64, device="cuda")
    d_own, d_opp = dev(np.asarray(own, np.uint64)), dev(np.asarray(opp, np.uint64))  # keep alive
    nat.check(nat.lib.oth_legal_gpu(nat.ptr(d_own), nat.ptr(d_opp), nat.ptr(out), n,
                                    nat.stream_ptr()), "oth_legal_gpu")
    torch.cuda.synchronize()
    return host_u64(out)


def own_opp(pos, neg, player):
    own = np.where(player == 1, pos, neg).astype(np.uint64)
    opp = np.where(player == 1, neg, pos).astype(np.uint64)
    return own, opp


def test_corpus_matches_reference_on_device():
    d = load_golden("board_corpus.npz")
    own, opp = own_opp(d["pos"], d["neg"], d["player"])
    assert (legal_gpu(own, opp) == d["valid"]).all()
    o, p, lg, st = step_gpu(own, opp, d["action"])
    nown, nopp = own_opp(d["npos"], d["nneg"], -d["player"])
    assert (o == nown).all() and (p == nopp).all()
    flags = st & 0xFF
    assert ((flags & 4) == 0).all()
    assert ((flags & 1) == d["term_next"]).all()
    assert (((flags & 8) != 0) == (d["action"] == 64)).all()
    score = nat.status_score(st)
    assert (score * -d["player"] == d["score_p1"]).all()
    term = d["term_next"] == 1
    assert (np.sign(score[term]) == d["val_next"][term]).all()
    assert (lg == legal_gpu(nown, nopp)).all()


def _random_positions(n, seed):
    """Reachable positions (random playouts) plus uniform random disjoint pairs."""
    rng = np.random.default_rng(seed)
    d = load_golden("board_corpus.npz")
    own, opp = own_opp(d["pos"], d["neg"], d["player"])
    idx = rng.integers(0, len(own), n // 2)
    a_own, a_opp = own[idx], opp[idx]
    occ = rng.integers(0, 2**63, n - n // 2, dtype=np.int64).astype(np.uint64) | \
        (rng.integers(0, 2, n - n // 2).astype(np.uint64) << np.uint64(63))
    col = rng.integers(0, 2**63, n - n // 2, dtype=np.int64).astype(np.uint64)
    b_own, b_opp = occ & col, occ & ~col
    own = np.concatenate([a_own, b_own])
    opp = np.concatenate([a_opp, b_opp])
    act = rng.integers(0, 65, n).astype(np.uint8)  # mostly illegal for the random half
    lgl = ob.legal_batch(own, opp)
    # for the reachable half pick a legal action (or pass)
    for i in range(n // 2):
        m = int(lgl[i])
        if m:
            bits = [b for b in range(64) if (m >> b) & 1]
            act[i] = bits[int(rng.integers(0, len(bits)))]
        else:
            act[i] = 64
    return own, opp, act


def test_step_matches_oracle_random_and_illegal():
    own, opp, act = _random_positions(1 << 16, 7)
    o, p, lg, st = step_gpu(own, opp, act)
    ro, rp, rl, rs, _ = ob.step_batch(own, opp, act)
    assert (o == ro).all() and (p == rp).all() and (lg == rl).all() and (st == rs).all()
    assert (legal_gpu(own, opp) == ob.legal_batch(own, opp)).all()
    assert (nat.status_flags(st) & 4).any()  # illegal placements were exercised


def test_step_large_batch_matches_cpu_entry_point():
    """2^22 positions (grid-stride path) against the host build of the same C ABI, and a
    checksum against the oracle on a strided subsample."""
    own, opp, act = _random_positions(1 << 18, 11)
    rep = 16
    own, opp, act = np.tile(own, rep), np.tile(opp, rep), np.tile(act, rep)
    o, p, lg, st = step_gpu(own, opp, act)
    co, cp, cl, cs = nat.step_cpu(own, opp, act, raise_illegal=False)
    assert (o == co).all() and (p == cp).all() and (lg == cl).all() and (st == cs).all()
    sub = slice(0, None, 97)
    ro, rp, rl, rs, _ = ob.step_batch(own[sub], opp[sub], act[sub])
    assert (o[sub] == ro).all() and (st[sub] == rs).all()


def test_step_odd_sizes_and_unaligned_buffers():
    """oth_step_gpu runs the paired kernel (two positions per lane, 16-byte accesses) on
    aligned buffers and the one-per-lane kernel otherwise: odd counts (the half-live last
    pair) and buffers offset by one element (unaligned: the fallback kernel), both
    bit-exact against the host build of the same entry point."""
    own, opp, act = _random_positions(1 << 17, 5)
    for n in (1, 2, 3, 255, 257, 4097, 65537):
        for off in (0, 1):
            t_own, t_opp, t_act = dev(own[:n + 1]), dev(opp[:n + 1]), dev(act[:n + 1])
            outs = [torch.zeros(n + 1, dtype=torch.int64, device="cuda") for _ in range(3)]
            st = torch.zeros(n + 1, dtype=torch.int16, device="cuda")
            sl = slice(off, off + n)
            nat.check(nat.lib.oth_step_gpu(*[nat.ptr(x[sl]) for x in (t_own, t_opp, t_act)],
                                           *[nat.ptr(x[sl]) for x in outs], nat.ptr(st[sl]), n,
                                           nat.stream_ptr()), "oth_step_gpu")
            torch.cuda.synchronize()
            co, cp, cl, cs = nat.step_cpu(own[sl], opp[sl], act[sl], raise_illegal=False)
            assert (host_u64(outs[0])[sl] == co).all(), (n, off)
            assert (host_u64(outs[1])[sl] == cp).all(), (n, off)
            assert (host_u64(outs[2])[sl] == cl).all(), (n, off)
            assert (st.cpu().numpy().view(np.uint16)[sl] == cs).all(), (n, off)
            # nothing written outside the n outputs
            other = n if off == 0 else 0
            assert host_u64(outs[0])[other] == 0 and st.cpu().numpy()[other] == 0, (n, off)


def test_empty_batch_and_edge_boards():
    assert step_gpu([], [], [])[0].size == 0
    full = np.array([0xFFFFFFFFFFFFFFFF], np.uint64)
    zero = np.array([0], np.uint64)
    o, p, lg, st = step_gpu(full, zero, [64])  # full board, pass
    assert lg[0] == 0 and nat.status_flags(st)[0] & 1
    assert nat.status_score(st)[0] == -64
    e = load_golden("edge_cases.npz")
    for black, white, mask, forb in e["wrap"]:
        assert legal_gpu(np.array([black]), np.array([white]))[0] == mask


def test_d4_device_matches_numpy_tables():
    d = load_golden("d4.npz")
    rng = np.random.default_rng(3)
    x = rng.integers(0, 2**63, 4096, dtype=np.int64).astype(np.uint64)
    sym = rng.integers(0, 8, 4096).astype(np.uint8)
    out = torch.empty(4096, dtype=torch.int64, device="cuda")
    d_x, d_sym = dev(x), dev(sym)  # keep the inputs alive across the async launch
    nat.check(nat.lib.oth_d4_gpu(nat.ptr(d_x), nat.ptr(d_sym), nat.ptr(out), 4096,
                                 nat.stream_ptr()), "oth_d4_gpu")
    torch.cuda.synchronize()
    got = host_u64(out)
    bits = ((x[:, None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).astype(np.uint8)
    for i in range(0, 4096, 7):
        # sym_board[s] = the index array transformed: out[j] = in[sym_board[s][j]]
        src = d["sym_board"][sym[i]]
        want = int(np.bitwise_or.reduce(
            bits[i][src].astype(np.uint64) << np.arange(64, dtype=np.uint64)))
        assert int(got[i]) == want
