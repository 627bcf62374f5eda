"""Replay-buffer aggregation on the GPU: a drop-in for the reference's
Trainer._aggregate_duplicates (train.py:142-173) and a device-tensor form for buffers that
already live in HBM (the engine's sample ring).

    states, policies, values = aggregate_duplicates(trainer.replay_buffer)

`replay_buffer` holds the reference's `(state int8 (8,8), pi float32 (65,), v float,
version int)` rows (train.py:136-140); the result is the reference's three aligned lists
(int8 states, float32 pi, np.float32 values) in its first-occurrence order, bit-exact
(tests/test_replay_gpu.py).  Rows are keyed on the canonical board as bitboards (own =
+1 stones, opp = -1 stones) instead of its SHA-1.
"""
import ctypes

import numpy as np
import torch

import az_native as nat


def aggregate_rows(own, opp, ver, pi, v):
    """Device tensors in, device tensors out: own/opp int64 [n] (bit patterns), ver int32
    [n], pi float32 [n, 65], v float64 [n] -> (own, opp, ver, pi, v float32, count) of the
    collapsed samples, in order of first occurrence."""
    n = int(own.shape[0])
    dev = own.device
    cont = lambda t, dt: t.to(device=dev, dtype=dt).contiguous()  # noqa: E731
    own, opp = cont(own, torch.int64), cont(opp, torch.int64)
    ver, pi, v = cont(ver, torch.int32), cont(pi, torch.float32).reshape(n, 65), cont(v, torch.float64)
    m = max(n, 1)
    out = {"own": torch.empty(m, dtype=torch.int64, device=dev),
           "opp": torch.empty(m, dtype=torch.int64, device=dev),
           "ver": torch.empty(m, dtype=torch.int32, device=dev),
           "pi": torch.empty(m, 65, dtype=torch.float32, device=dev),
           "v": torch.empty(m, dtype=torch.float32, device=dev),
           "count": torch.empty(m, dtype=torch.int32, device=dev)}
    n_out = torch.zeros(1, dtype=torch.int32, device=dev)
    wsb = ctypes.c_size_t(0)
    args = [nat.ptr(own), nat.ptr(opp), nat.ptr(ver), nat.ptr(pi), nat.ptr(v), n,
            nat.ptr(out["own"]), nat.ptr(out["opp"]), nat.ptr(out["ver"]), nat.ptr(out["pi"]),
            nat.ptr(out["v"]), nat.ptr(out["count"]), nat.ptr(n_out)]
    nat.check(nat.lib.az_replay_aggregate_gpu(*args, None, ctypes.addressof(wsb),
                                              nat.stream_ptr()), "az_replay_aggregate_gpu")
    ws = torch.empty(max(int(wsb.value), 1), dtype=torch.uint8, device=dev)
    nat.check(nat.lib.az_replay_aggregate_gpu(*args, nat.ptr(ws), ctypes.addressof(wsb),
                                              nat.stream_ptr()), "az_replay_aggregate_gpu")
    k = int(n_out.item())
    return {key: t[:k] for key, t in out.items()}


def aggregate_duplicates(replay_buffer, device=None):
    """Trainer._aggregate_duplicates (train.py:142-173) on the GPU: same inputs, same three
    lists, same order, same values."""
    rows = list(replay_buffer)
    if not rows:
        return [], [], []
    device = torch.device(device or "cuda")
    states = np.stack([np.asarray(r[0], np.int8).reshape(64) for r in rows])
    own, opp = nat.pack_np(states, np.ones(len(rows), np.int8))
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(device=device, dtype=dt)  # noqa: E731
    res = aggregate_rows(t(own.view(np.int64), torch.int64), t(opp.view(np.int64), torch.int64),
                         t(np.array([r[3] for r in rows], np.int32), torch.int32),
                         t(np.stack([np.asarray(r[1], np.float32) for r in rows]), torch.float32),
                         t(np.array([float(r[2]) for r in rows], np.float64), torch.float64))
    o_own = res["own"].cpu().numpy().view(np.uint64)
    o_opp = res["opp"].cpu().numpy().view(np.uint64)
    boards = nat.unpack_np(o_own, o_opp, np.ones(len(o_own), np.int8)).reshape(-1, 8, 8)
    pis = res["pi"].cpu().numpy()
    vs = res["v"].cpu().numpy()
    return ([boards[i].copy() for i in range(len(boards))],
            [pis[i].copy() for i in range(len(pis))],
            [np.float32(x) for x in vs])
