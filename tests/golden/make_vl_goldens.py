"""Golden vectors for the multi-leaf (virtual-loss) search, made by running the REFERENCE's
own threaded simulation code under a controlled thread schedule.  Build container only
(imports /root/reference read-only); writes tests/golden/mcts_vl_cases.npz.

The reference searches with args['num_threads'] worker threads (MCTS_model.py:196-197,
:237-242), each running MCTS._simulate (:372-395): walk down adding a virtual loss to every
node passed (Node.add_virtual_loss, :115-118; Node.value and _get_ucb_score count it,
:110-139), back a terminal value up at once, or evaluate + expand + back up an unexpanded
leaf, then revert the path's virtual loss.  Its thread interleaving is up to the OS, so the
search is nondeterministic.  The engine's `leaves_per_step = K` mode is one fixed legal
interleaving of it, and this script forces exactly that interleaving on the reference:

    repeat until num_simulations are done:
        start simulations one at a time, each on its own thread; wait until it either
        finished (terminal leaf: backed up, virtual loss reverted) or is blocked inside
        policy.inference (an unexpanded leaf: its path's virtual loss stays applied);
        stop when K are blocked or the remaining simulations are all started;
        release the blocked ones in start order, each running to completion (expand,
        back up, revert) before the next is released.

Two simulations blocked on the same leaf both expand it (the second replaces the children
with identical fresh ones -- nothing visited them in between) and both back up its value:
the engine expands once and backs up twice, the same tree.  The root expansion, tree reuse
(make_move) and pi (policy_improve_step with no further simulations) are the reference's
own code.  Policy: the deterministic mock (tests/mock_policy.py).

    python tests/golden/make_vl_goldens.py
"""
import os
import sys
import threading
import time

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True

import numpy as np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_goldens import RngRecorder, bb_from_state, encode_log, random_position  # noqa: E402
from mock_policy import MockPolicy  # noqa: E402


class GatedPolicy:
    """MockPolicy whose inference blocks worker threads until the driver releases them."""

    def __init__(self):
        self.inner = MockPolicy()
        self.cv = threading.Condition()
        self.blocked = set()   # thread idents waiting inside inference
        self.released = set()

    def inference(self, state, player):
        out = self.inner.inference(state, player)
        me = threading.get_ident()
        if threading.current_thread() is threading.main_thread():
            return out  # the root expansion (policy_improve_step) runs unblocked
        with self.cv:
            self.blocked.add(me)
            self.cv.notify_all()
            self.cv.wait_for(lambda: me in self.released)
            self.released.discard(me)
            self.blocked.discard(me)
        return out


def controlled_simulations(m, policy, sims, K):
    """Run `sims` reference simulations with at most K blocked on inference at a time."""
    done = 0
    while done < sims:
        pending = []
        while done + len(pending) < sims and len(pending) < K:
            t = threading.Thread(target=m._simulate, args=(m.root,))
            t.start()
            with policy.cv:
                policy.cv.wait_for(lambda: t.ident in policy.blocked or not t.is_alive(),
                                   timeout=60)
                blocked = t.ident in policy.blocked
            if blocked:
                pending.append(t)
            else:
                t.join()
                done += 1
        for t in pending:
            with policy.cv:
                policy.released.add(t.ident)
                policy.cv.notify_all()
            t.join()
            done += 1


def gen_vl():
    from envs.othello import OthelloGameNew
    from MCTS_model import MCTS, Node

    g = OthelloGameNew(8)
    rng = np.random.default_rng(29)
    specs = [random_position(g, rng, plies) for plies in (0, 6, 14, 22, 30, 38, 46, 54)]
    rows = dict(pos=[], neg=[], player=[], sims=[], k=[], c_puct=[], eps=[], moves=[],
                counts=[], root_value=[], probs=[], root_n=[], log_case=[])
    logs = []
    case_id = 0
    for si, (state, player) in enumerate(specs):
        for sims, K, cp, eps in ((100, 4, 2.0, 0.0), (100, 2, 1.0, 0.3), (400, 4, 2.0, 0.3),
                                 (200, 8, 2.0, 0.0)):
            if sims == 400 and si % 2:
                continue
            np.random.seed(500 + case_id)
            args = {"c_puct": cp, "num_simulations": sims, "num_threads": K}
            policy = GatedPolicy()
            m = MCTS(g, args, policy, dirichlet_alpha=1.0, dirichlet_epsilon=eps)
            st, pl = state.copy(), player
            with RngRecorder() as rec:
                for mv in range(2):
                    # policy_improve_step (MCTS_model.py:217-235) up to its simulations
                    if m.root is None:
                        m.root = Node(env=g, args=args, state=st.copy(), player=pl, action=None)
                    if m.root.is_leaf():
                        m._expand_and_evaluate(m.root)
                    controlled_simulations(m, policy, sims, K)
                    # ... and its pi from the counts (no further simulations)
                    m.args = dict(args, num_simulations=0)
                    probs = m.policy_improve_step(st, pl, temp=1.0)
                    m.args = args
                    counts = np.zeros(65, np.int64)
                    for a, ch in m.root.children.items():
                        counts[a] = ch.visit_count
                        assert ch.virtual_visits == 0
                    p, n = bb_from_state(st)
                    rows["pos"].append(p)
                    rows["neg"].append(n)
                    rows["player"].append(pl)
                    rows["sims"].append(sims)
                    rows["k"].append(K)
                    rows["c_puct"].append(cp)
                    rows["eps"].append(eps)
                    rows["moves"].append(mv)
                    rows["counts"].append(counts)
                    rows["root_value"].append(float(m.root.value))
                    rows["probs"].append(np.asarray(probs, np.float32))
                    rows["root_n"].append(m.root.visit_count)
                    rows["log_case"].append(case_id)
                    a = int(np.argmax(counts))
                    nxt = g.get_next_state(st, a, pl)
                    if g.get_value_and_terminated(nxt, a, pl)[1]:
                        break
                    m.make_move(a)
                    st, pl = nxt, -pl
            m.pool.shutdown()
            kinds, _, _, noise = encode_log(rec.log)
            assert (kinds == 0).all(), "only Dirichlet draws at temperature 1"
            logs.append(noise)
            case_id += 1
    out = {}
    for k in ("pos", "neg"):
        out[k] = np.array(rows[k], np.uint64)
    for k in ("player", "sims", "k", "moves", "root_n", "log_case"):
        out[k] = np.array(rows[k], np.int64)
    for k in ("c_puct", "eps", "root_value"):
        out[k] = np.array(rows[k], np.float64)
    out["counts"] = np.array(rows["counts"], np.int64)
    out["probs"] = np.array(rows["probs"], np.float32)
    out["n_cases"] = np.int64(case_id)
    offs = [0]
    for nz in logs:
        offs.append(offs[-1] + len(nz))
    out["noise_offsets"] = np.array(offs, np.int64)
    out["noise"] = np.concatenate(logs) if offs[-1] else np.zeros((0, 65))
    np.savez_compressed(os.path.join(HERE, "mcts_vl_cases.npz"), **out)
    print("mcts_vl_cases:", case_id, "cases,", len(out["pos"]), "searches")


if __name__ == "__main__":
    t0 = time.time()
    gen_vl()
    print(f"{time.time() - t0:.1f}s")
