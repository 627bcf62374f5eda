"""TEST INFRASTRUCTURE ONLY — sequential restatement of the reference MCTS.

Restates MCTS_model.py (Node :46-169, MCTS :172-395) for args['num_threads'] = 1, the
deterministic mode of the reference, on a flat tree of bitboards.
Every float operation reproduces the reference's NumPy-2 (NEP 50) promotion explicitly:

  * node value  = W / N in float64, 0.0 when unvisited          (MCTS_model.py:110-114)
  * PUCT        = float32(-value) + u, u = ((c*P) * sqrt(Np+1+1e-8)) / (1+Nc) in float32,
                  where the parent's own virtual visit (+1) is counted    (:129-139, :378)
                  and the whole score is float64 when P is float64 (Dirichlet-noised root)
  * argmax over children in ascending action, first maximum wins          (:362-370)
  * priors *= valid_mask; sum (NumPy pairwise); /= sum if > 1e-12          (:345-349)
  * Dirichlet noise (1-eps)*P + eps*noise only when the root itself is expanded (:340-343)
  * backup alternates sign from the leaf to the root                     (:160-169)
  * pi from child visit counts                                           (:244-274)

leaves_per_step = K > 1 restates the reference's threaded search (args['num_threads'] = K,
:196-197, :237-242, :372-395) in the one fixed interleaving the engine implements and
tests/golden/make_vl_goldens.py forces on the reference: simulations start one at a time;
each adds a virtual loss to every node it passes (:115-118) -- Node.value = (W + VV) / (N + VV),
PUCT counts the parent's and children's virtual visits (:110-139); a terminal one backs up
at once; one reaching an unexpanded leaf waits (its virtual loss stays) until K wait or the
simulations are all started; the waiting ones then finish in start order (expand once per
distinct leaf, back up each one's value).

RNG draws go through an adapter so a test can either replay the reference's global
np.random stream call-for-call (NumpyRng) or inject recorded draws (LogRng).
"""
import math

import numpy as np

from . import board as ob


class NumpyRng:
    """Consumes np.random exactly as the reference does."""

    def dirichlet(self, alpha, n):
        return np.random.dirichlet([alpha] * n)

    def choice_tie(self, best):
        return np.random.choice(best)

    def choice_p(self, n, p):
        return np.random.choice(n, p=p)


class LogRng:
    """Replays draws recorded by tests/golden/make_goldens.py (RngRecorder)."""

    def __init__(self, kinds, a, b, noise):
        self.kinds, self.a, self.b, self.noise = list(kinds), list(a), list(b), noise
        self.i = 0

    def _next(self, kind):
        k = self.kinds[self.i]
        assert k == kind, f"rng log mismatch at {self.i}: want {kind}, have {k}"
        a, b = self.a[self.i], self.b[self.i]
        self.i += 1
        return a, b

    def dirichlet(self, alpha, n):
        a, _ = self._next(0)
        return np.array(self.noise[int(a)], np.float64)

    def choice_tie(self, best):
        k, j = self._next(1)
        assert int(k) == len(best)
        return best[int(j)]

    def choice_p(self, n, p):
        u, _ = self._next(2)
        cdf = np.asarray(p, np.float64).cumsum()
        cdf /= cdf[-1]
        return int(cdf.searchsorted(u, side="right"))


def ucb_scores(prior, n_child, w_child, n_parent, c_puct, vv_parent=1, vv_child=None):
    """PUCT of every child (MCTS_model.py:129-139) with the parent's virtual visits (its
    own +1 during the descent, plus those of waiting simulations) and the children's."""
    out = []
    sq = math.sqrt(n_parent + vv_parent + 1e-8)
    vv_child = vv_child or [0] * len(prior)
    for p, n, w, vv in zip(prior, n_child, w_child, vv_child):
        q = -(0.0 if n + vv == 0 else (w + float(vv)) / (n + vv))
        if isinstance(p, np.float64):
            u = c_puct * float(p) * sq / (1 + n + vv)
            out.append(q + u)
        else:
            u = np.float32(np.float32(np.float32(np.float32(c_puct) * p) * np.float32(sq))
                           / np.float32(1 + n + vv))
            out.append(np.float32(np.float32(q) + u))
    return out


class SeqMCTS:
    """Flat-array tree; node 0 is the root after every re-root."""

    def __init__(self, c_puct, num_simulations, evaluate=None, dirichlet_alpha=0.03,
                 dirichlet_epsilon=0.0, rng=None, leaves_per_step=1):
        self.c_puct = c_puct
        self.K = max(1, int(leaves_per_step))
        self.sims = num_simulations
        self.evaluate = evaluate  # (own, opp, player) -> (priors f32[65], value float)
        self.alpha = dirichlet_alpha
        self.eps = dirichlet_epsilon
        self.rng = rng or NumpyRng()
        self.reset()

    # ---- tree storage -------------------------------------------------------------
    def reset(self):
        self.own, self.opp, self.player, self.legal = [], [], [], []
        self.N, self.W, self.prior, self.parent, self.action = [], [], [], [], []
        self.kids = []  # list of child indices (ascending action)
        self.term, self.tval = [], []
        self.root = -1

    def _new(self, own, opp, player, parent, action, prior, is_root):
        i = len(self.own)
        lg = ob.legal(own, opp)
        self.own.append(own)
        self.opp.append(opp)
        self.player.append(player)
        self.legal.append(lg)
        self.N.append(0)
        self.W.append(0.0)
        self.prior.append(prior)
        self.parent.append(parent)
        self.action.append(action)
        self.kids.append([])
        if is_root:
            t, v = False, 0
        elif lg or ob.legal(opp, own):
            t, v = False, 0
        else:
            d = ob.popc(own) - ob.popc(opp)
            t, v = True, (1 if d > 0 else (-1 if d < 0 else 0))
        self.term.append(t)
        self.tval.append(v)
        return i

    def valid_actions(self, i):
        lg = self.legal[i]
        return [a for a in range(64) if (lg >> a) & 1] or [64]

    def value(self, i):
        return 0.0 if self.N[i] == 0 else self.W[i] / self.N[i]

    # ---- search ---------------------------------------------------------------------
    def set_root(self, own, opp, player):
        self.reset()
        self.root = self._new(own, opp, player, -1, None, 0.0, True)

    def _backup(self, i, v):
        s = 1
        while i >= 0:
            self.N[i] += 1
            self.W[i] += s * v
            s = -s
            i = self.parent[i]

    def _rollout(self, own, opp):
        """MCTS._rollout (MCTS_model.py:276-303) with the reference's np.random draws."""
        side = 1
        while True:
            lg = ob.legal(own, opp)
            acts = [a for a in range(64) if (lg >> a) & 1] or [64]
            a = int(np.random.choice(np.array(acts)))
            own, opp = ob.make_move(own, opp, a)
            side = -side
            if not ob.legal(own, opp) and not ob.legal(opp, own):
                d = (ob.popc(own) - ob.popc(opp)) * side
                return 1 if d > 0 else (-1 if d < 0 else 0)

    def _expand(self, i):
        self._backup(i, self._expand_only(i))

    def _expand_only(self, i):
        if self.evaluate is None:
            priors = np.ones(65, np.float32)
            v = self._rollout(self.own[i], self.opp[i])
        else:
            priors, v = self.evaluate(self.own[i], self.opp[i], self.player[i])
            priors = np.array(priors, np.float32)
        if i == self.root and self.eps > 0:
            noise = self.rng.dirichlet(self.alpha, len(priors))
            priors = (1 - self.eps) * priors + self.eps * noise
        valid = np.zeros(65, np.uint8)
        acts = self.valid_actions(i)
        valid[acts] = 1
        priors = priors * valid
        tot = priors.sum()
        if tot > 1e-12:
            priors = priors / tot
        for a in acts:
            own, opp = ob.make_move(self.own[i], self.opp[i], a)
            c = self._new(own, opp, -self.player[i], i, a, priors[a], False)
            self.kids[i].append(c)
        return v

    def _select(self, i):
        kids = self.kids[i]
        sc = ucb_scores([self.prior[k] for k in kids], [self.N[k] for k in kids],
                        [self.W[k] for k in kids], self.N[i], self.c_puct)
        best = 0
        for j in range(1, len(kids)):
            if sc[j] > sc[best]:
                best = j
        return kids[best]

    def simulate(self):
        i = self.root
        while True:
            if self.term[i]:
                self._backup(i, self.tval[i])
                return
            if not self.kids[i]:
                self._expand(i)
                return
            i = self._select(i)

    def _select_vl(self, i, vv):
        kids = self.kids[i]
        sc = ucb_scores([self.prior[k] for k in kids], [self.N[k] for k in kids],
                        [self.W[k] for k in kids], self.N[i], self.c_puct,
                        1 + vv.get(i, 0), [vv.get(k, 0) for k in kids])
        best = 0
        for j in range(1, len(kids)):
            if sc[j] > sc[best]:
                best = j
        return kids[best]

    def simulate_batch(self, remaining):
        """One batch of the K-leaf search (simulations started one after another until K wait
        on the evaluation or none remain; the interleaving make_vl_goldens.py forces on the
        reference's workers): returns the simulations it completed."""
        done, pending, vv = 0, [], {}
        while done + len(pending) < remaining and len(pending) < self.K:
            i, path = self.root, []
            while True:
                path.append(i)
                if self.term[i]:
                    self._backup(i, self.tval[i])
                    done += 1
                    break
                if not self.kids[i]:
                    pending.append(i)
                    for n in path:
                        vv[n] = vv.get(n, 0) + 1
                    break
                i = self._select_vl(i, vv)
        values = {}
        for leaf in pending:
            if leaf not in values:
                values[leaf] = self._expand_only(leaf)
            self._backup(leaf, values[leaf])
            done += 1
        return done

    def search(self, own, opp, player, temp=1.0):
        """policy_improve_step (MCTS_model.py:217-274)."""
        if self.root < 0:
            self.set_root(own, opp, player)
        else:
            assert self.own[self.root] == own and self.opp[self.root] == opp
            assert self.player[self.root] == player
        if not self.kids[self.root]:
            self._expand(self.root)
        if self.K == 1:
            for _ in range(self.sims):
                self.simulate()
        else:
            done = 0
            while done < self.sims:
                done += self.simulate_batch(self.sims - done)
        counts = np.zeros(65, np.float32)
        for k in self.kids[self.root]:
            counts[self.action[k]] = self.N[k]
        if abs(temp) < 0.1:
            best = np.where(counts == counts.max())[0]
            pick = self.rng.choice_tie(best)
            probs = np.zeros_like(counts)
            probs[pick] = 1.0
            return probs
        ce = counts ** (1.0 / temp)
        norm = np.sum(ce)
        if norm < 1e-12:
            acts = self.valid_actions(self.root)
            probs = np.zeros(65, np.float32)
            probs[acts] = 1.0 / len(acts)
            return probs
        return ce / norm

    def root_counts(self):
        c = np.zeros(65, np.int64)
        for k in self.kids[self.root]:
            c[self.action[k]] = self.N[k]
        return c

    def make_move(self, action):
        """MCTS.make_move (MCTS_model.py:200-215): keep the chosen subtree, compacted."""
        if self.root < 0:
            return
        new = None
        for k in self.kids[self.root]:
            if self.action[k] == action:
                new = k
        if new is None:
            raise KeyError(action)
        old = {f: getattr(self, f) for f in ("own", "opp", "player", "legal", "N", "W",
                                             "prior", "action", "term", "tval")}
        oldkids = self.kids
        self.reset()
        order, remap, q = [], {}, [new]
        while q:  # BFS copy, children stay contiguous and ascending
            x = q.pop(0)
            remap[x] = len(order)
            order.append(x)
            q.extend(oldkids[x])
        for x in order:
            for f, arr in old.items():
                getattr(self, f).append(arr[x])
            self.kids.append([remap[k] for k in oldkids[x]])
            self.parent.append(-1)
        for x in order:
            for k in oldkids[x]:
                self.parent[remap[k]] = remap[x]
        self.root = 0
