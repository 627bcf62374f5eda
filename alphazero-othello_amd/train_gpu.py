"""The training side of a generation on the GPU: the Trainer's DataLoader
over RandomSymmetryDataset (reference train.py:26-42, 175-200) as a device-resident batch
iterator with the random dihedral augmentation of get_random_symmetry (envs/othello.py:
501-526) applied per sample by the bitboard D4 kernel (oth_d4_gpu) and a permutation
gather on pi, and Trainer.train_iters' loss and update (train.py:261-301) on those
batches.

Each sample's symmetry is sym = k + 4*flip (rot90 k times, then fliplr) drawn from a torch
generator instead of NumPy's global RNG; for a given (k, flip) the augmented state and pi
equal the reference's bit for bit (tests/test_train_gpu.py, fixture from the reference).
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

import az_native as nat

_SQ = torch.arange(64, dtype=torch.int64)


def pi_source_tables():
    """int64 [8, 65]: pi_out[i] = pi[src[sym, i]] (index 64, the pass, maps to itself)."""
    src = np.empty((8, 65), np.int64)
    single = (np.uint64(1) << np.arange(64, dtype=np.uint64))
    for s in range(8):
        moved = nat.d4_cpu(single, s)  # square j's stone lands on square dst[j]
        dst = np.array([int(m).bit_length() - 1 for m in moved], np.int64)
        src[s, dst] = np.arange(64)
        src[s, 64] = 64
    return src


def augment(own, opp, pi, sym):
    """own/opp int64 [B] canonical bitboards (own = +1 stones), pi float32 [B, 65], sym int
    [B] in 0..7 -> (state float32 [B, 1, 8, 8], pi float32 [B, 65]) transformed like
    get_random_symmetry with k = sym & 3, flip = sym >> 2."""
    dev = own.device
    B = own.shape[0]
    sym8 = sym.to(torch.uint8).contiguous()
    o2 = torch.empty_like(own)
    p2 = torch.empty_like(opp)
    for src, dst in ((own.contiguous(), o2), (opp.contiguous(), p2)):
        nat.check(nat.lib.oth_d4_gpu(nat.ptr(src), nat.ptr(sym8), nat.ptr(dst), B,
                                     nat.stream_ptr()), "oth_d4_gpu")
    sq = _SQ.to(dev)
    state = (((o2[:, None] >> sq) & 1) - ((p2[:, None] >> sq) & 1)).to(torch.float32)
    tables = getattr(augment, "_tables", {}).get(dev)
    if tables is None:
        tables = torch.from_numpy(pi_source_tables()).to(dev)
        augment._tables = {**getattr(augment, "_tables", {}), dev: tables}
    pi_out = torch.gather(pi, 1, tables[sym.to(torch.int64)])
    return state.view(B, 1, 8, 8), pi_out


class DeviceReplayLoader:
    """(state [B,1,8,8], pi [B,65], v [B,1]) float32 batches from aggregated samples held in
    HBM, shuffled and D4-augmented per sample — the reference's
    DataLoader(RandomSymmetryDataset(...), shuffle=True)."""

    def __init__(self, states, policies, values, batch_size, shuffle=True, augment=True,
                 device="cuda", seed=None):
        self.device = torch.device(device)
        st = np.asarray(np.stack([np.asarray(s).reshape(64) for s in states]), np.float32)
        own, opp = nat.pack_np(np.rint(st).astype(np.int8), np.ones(len(st), np.int8))
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(self.device, dt)  # noqa: E731
        self.own = t(own.view(np.int64), torch.int64)
        self.opp = t(opp.view(np.int64), torch.int64)
        self.pi = t(np.stack([np.asarray(p, np.float32) for p in policies]), torch.float32)
        self.v = t(np.asarray(values, np.float32).reshape(-1, 1), torch.float32)
        self.batch_size, self.shuffle, self.aug = int(batch_size), shuffle, augment
        self.gen = torch.Generator(device=self.device)
        if seed is not None:
            self.gen.manual_seed(int(seed))

    def __len__(self):
        return (self.own.shape[0] + self.batch_size - 1) // self.batch_size

    def __iter__(self):
        n = self.own.shape[0]
        order = (torch.randperm(n, generator=self.gen, device=self.device) if self.shuffle
                 else torch.arange(n, device=self.device))
        for b in range(0, n, self.batch_size):
            idx = order[b:b + self.batch_size]
            sym = (torch.randint(0, 8, (idx.shape[0],), generator=self.gen, device=self.device)
                   if self.aug else torch.zeros(idx.shape[0], dtype=torch.int64, device=self.device))
            s, p = augment(self.own[idx], self.opp[idx], self.pi[idx], sym)
            yield s, p, self.v[idx]


def train_iters(policy, optimizer, loader, entropy_coef, value_loss=None):
    """One pass of Trainer.train_iters (train.py:261-301) over device batches: policy
    cross-entropy + MSE value loss - entropy bonus, grad-norm clip 5.0.  Returns the
    average policy, value and entropy terms."""
    value_loss = value_loss or nn.MSELoss()
    policy.train()
    tp = tv = te = 0.0
    nb = 0
    for state, target_pi, target_v in loader:
        logits, value = policy(state)
        log_probs = F.log_softmax(logits, dim=-1)
        p_loss = -torch.mean(torch.sum(target_pi * log_probs, dim=-1))
        probs = torch.softmax(logits, dim=-1)
        entropy = torch.mean(torch.sum(-probs * log_probs, dim=-1))
        e_loss = -entropy_coef * entropy
        v_loss = value_loss(value, target_v)
        loss = p_loss + v_loss + e_loss
        optimizer.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(policy.parameters(), 5.0)
        optimizer.step()
        tp += float(p_loss.detach())
        tv += float(v_loss.detach())
        te += float(-e_loss.detach())
        nb += 1
    return tp / max(nb, 1), tv / max(nb, 1), te / max(nb, 1)
