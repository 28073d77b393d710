"""Canonical host view of one Splendor table, shared by the fixture generator and the tests.

The view mirrors the reference ``SplendorState`` (engine/state.py:74-104) with plain ints:
card ids 0..89 (JSON order, engine/state.py:121-142), noble indices 0..9 (reference id − 1000,
engine/state.py:160-174), -1 for an empty board slot / taken noble / ``winner_index is None``.

It is the same record as ``spl_table_t`` (include/splendor_table.h): the C oracle and the device
download produce it, so trajectories can be compared field by field and by digest.

Test infrastructure only — nothing here is imported by the product package.
"""
import hashlib
import json

MAXP = 4


def empty_view(P):
    return dict(
        P=P,
        bank=[0] * 6,
        players=[dict(tokens=[0] * 6, bonuses=[0] * 5, prestige=0, reserved=[], revealed=[],
                      nobles=[]) for _ in range(P)],
        board=[-1] * 12,
        decks=[[], [], []],
        nobles=[],
        to_play=0, turn_count=1, move_count=0, game_over=0, winner=-1, turn_limit_reached=0,
    )


def canon(view):
    """Canonical bytes of a view.  Player noble lists are compared as sets: the device keeps the
    owner of each visible noble slot rather than acquisition order."""
    v = dict(view)
    v["players"] = []
    for p in view["players"]:
        q = dict(p)
        q["nobles"] = sorted(p["nobles"])
        q["revealed"] = [int(bool(x)) for x in p["revealed"]]
        v["players"].append(q)
    for k in ("game_over", "turn_limit_reached"):
        v[k] = int(bool(v[k]))
    return json.dumps(v, sort_keys=True, separators=(",", ":")).encode()


def digest(view):
    """64-bit digest of ``canon(view)`` (first 8 bytes of blake2b)."""
    return int.from_bytes(hashlib.blake2b(canon(view), digest_size=8).digest(), "little")


def from_ref_state(s):
    """Reference SplendorState -> view (used only by make_golden.py, which imports the reference)."""
    return dict(
        P=s.num_players,
        bank=[int(x) for x in s.bank],
        players=[dict(tokens=[int(x) for x in p.tokens], bonuses=[int(x) for x in p.bonuses],
                      prestige=int(p.prestige), reserved=[c.id for c in p.reserved],
                      revealed=[bool(x) for x in p.revealed_reserved],
                      nobles=[n.id - 1000 for n in p.nobles]) for p in s.players],
        board=[(c.id if c is not None else -1) for t in (1, 2, 3) for c in s.board[t]],
        decks=[[c.id for c in s.decks[t]] for t in (1, 2, 3)],
        nobles=[(n.id - 1000 if n is not None else -1) for n in s.nobles],
        to_play=int(s.to_play), turn_count=int(s.turn_count), move_count=int(s.move_count),
        game_over=int(bool(s.game_over)),
        winner=(-1 if s.winner_index is None else int(s.winner_index)),
        turn_limit_reached=int(bool(s.turn_limit_reached)),
    )
