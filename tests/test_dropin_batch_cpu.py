"""one_self_play's per-process batch on the host side (self_play_worker.py): the order games
are handed out in, and the batch size at train.py's settings (no GPU needed)."""
import numpy as np

import self_play_worker as spw

INIT_OWN, INIT_OPP = 0x0000000810000000, 0x0000001008000000


def _game_rows(slot, length, tag):
    """`length` sample rows of one synthetic game: the initial position, then positions with
    more stones (distinct per game through `tag`)."""
    own = [INIT_OWN] + [INIT_OWN | (1 << (i % 20)) | (1 << 40) for i in range(1, length)]
    opp = [INIT_OPP] + [INIT_OPP | (1 << (45 + tag)) for _ in range(1, length)]
    pi = np.zeros((length, 65), np.float32)
    pi[:, tag] = 1.0
    return {"own": np.array(own, np.uint64), "opp": np.array(opp, np.uint64), "pi": pi,
            "z": np.full(length, 0.25 * tag), "player": np.ones(length, np.int8),
            "slot": np.full(length, slot, np.int32)}


def _ring(games):
    return {k: np.concatenate([g[k] for g in games]) for k in games[0]}


def test_games_handed_out_in_slot_order_not_completion_order():
    """The sample ring is in completion order (the shortest game of a batch first); the
    batch is handed out in slot order, so which games a worker returns does not depend on
    their lengths (length-biased replay data)."""
    # completion order: slot 2 (shortest) .. slot 0 (longest)
    ring = _ring([_game_rows(2, 9, 2), _game_rows(3, 12, 3), _game_rows(1, 20, 1),
                  _game_rows(0, 31, 0)])
    games = spw._games_from_rows(ring)
    assert [len(g) for g in games] == [31, 20, 9, 12]
    for slot, g in enumerate(games):
        assert int(np.argmax(g[0][1])) == slot and g[0][2] == 0.25 * slot
        s0 = g[0][0]
        assert (s0 != 0).sum() == 4
    # rows without slot ids keep ring order (the old layout)
    ring.pop("slot")
    assert [len(g) for g in spw._games_from_rows(ring)] == [9, 12, 20, 31]


def test_batch_size_follows_the_workers_share(monkeypatch):
    monkeypatch.delenv("AZ_DROPIN_BATCH", raising=False)
    assert spw._dropin_batch_size() == 32
    # train.py's defaults: 300 games over os.cpu_count() workers
    assert spw._dropin_batch_size({"num_self_play": 300, "num_workers": 256}) == 2
    assert spw._dropin_batch_size({"num_self_play": 300, "num_workers": 8}) == 32
    assert spw._dropin_batch_size({"num_self_play": 100, "num_workers": 200}) == 1
    assert spw._dropin_batch_size({"c_puct": 2.0}) == 32
    monkeypatch.setenv("AZ_DROPIN_BATCH", "1")  # one game per call via the MCTS drop-in
    assert spw._dropin_batch_size({"num_self_play": 300, "num_workers": 8}) == 1
