"""Constants, game data and the HOST VIEW of one table.

The live state of every table is on the GPU (word planes in HBM, see csrc/spl_layout.h).  This
module gives the reference-shaped host view used for inspection, rendering and crafted-state
tests — the device copy is exchanged through spl_table_download / spl_table_upload.

Mirrors the reference's splendor_gym/engine/state.py:10-104 (colour order, DEFAULT_BANK, Card,
Noble, PlayerState, SplendorState field names) so code that reads ``env.state`` keeps working.
"""
import json
import os
from dataclasses import dataclass, field
from types import MappingProxyType
from typing import Dict, List, Optional

import numpy as np

TOKEN_COLORS = ["white", "blue", "green", "red", "black", "gold"]
STANDARD_COLORS = TOKEN_COLORS[:-1]
COLOR_INDEX = {c: i for i, c in enumerate(TOKEN_COLORS)}
STANDARD_COLOR_INDEX = {c: i for i, c in enumerate(STANDARD_COLORS)}
HUMAN_TO_INTERNAL = {"diamond": "white", "sapphire": "blue", "emerald": "green", "ruby": "red", "onyx": "black"}
INTERNAL_TO_HUMAN = {v: k for k, v in HUMAN_TO_INTERNAL.items()}
DEFAULT_BANK = {"white": 4, "blue": 4, "green": 4, "red": 4, "black": 4, "gold": 5}

DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")


def load_tables():
    """(cards int32[90, 8], nobles int32[10, 6]) from data/tables.json (tools/gen_tables.py)."""
    with open(os.path.join(DATA_DIR, "tables.json")) as f:
        t = json.load(f)
    cards = np.ascontiguousarray(np.array(t["cards"], np.int32))
    nobles = np.ascontiguousarray(np.array(t["nobles"], np.int32))
    assert cards.shape == (90, 8) and nobles.shape == (10, 6)
    return cards, nobles


@dataclass
class Card:
    """A card of one state (state.py:36-42).  Like the reference's (which initial_state loads afresh
    for every game), each host view holds its own Card objects, so a test may edit one in place
    (``card.cost = {...}``, tests/test_afford_nobles_obs.py:16-17): the edited fields reach the device
    as a card table of that state (SplendorState.card_table, evaluated on a context built from it)."""
    id: int
    tier: int
    color: str
    points: int
    cost: Dict[str, int]


@dataclass(frozen=True)
class Noble:
    id: int
    requirements: Dict[str, int]
    points: int = 3


_CARDS = None
_NOBLES = None
_CARD_ROWS = None


def cards_by_id():
    """The canonical cards (shared, read-only by convention): use card_copy() for a state's own."""
    global _CARDS, _NOBLES, _CARD_ROWS
    if _CARDS is None:
        c, n = load_tables()
        _CARD_ROWS = c
        _CARDS = [Card(i, int(r[0]), STANDARD_COLORS[int(r[1])], int(r[2]),
                       MappingProxyType({STANDARD_COLORS[k]: int(r[3 + k]) for k in range(5) if r[3 + k]}))
                  for i, r in enumerate(c)]
        _NOBLES = [Noble(1000 + i, MappingProxyType({STANDARD_COLORS[k]: int(r[k]) for k in range(5) if r[k]}),
                         int(r[5])) for i, r in enumerate(n)]
    return _CARDS


def card_copy(i):
    """A fresh, editable Card with the canonical data of card id `i`."""
    c = cards_by_id()[i]
    return Card(c.id, c.tier, c.color, c.points, dict(c.cost))


def card_row(card):
    """The device table row [tier, colour, points, cost w,b,g,r,k] of a Card's current fields."""
    return [int(card.tier), STANDARD_COLORS.index(card.color), int(card.points)] + \
        [int(card.cost.get(c, 0)) for c in STANDARD_COLORS]


def canonical_card_rows():
    cards_by_id()
    return _CARD_ROWS


def nobles_by_index():
    cards_by_id()
    return _NOBLES


@dataclass
class PlayerState:
    tokens: List[int] = field(default_factory=lambda: [0] * 6)
    bonuses: List[int] = field(default_factory=lambda: [0] * 5)
    prestige: int = 0
    reserved: List[Card] = field(default_factory=list)
    revealed_reserved: List[bool] = field(default_factory=list)
    nobles: List[Noble] = field(default_factory=list)

    def can_afford(self, card):
        """(affordable, discounted cost per colour) — state.py:61-71: colour tokens pay what the
        bonuses leave, gold covers the rest."""
        need, gold = [], 0
        for i, c in enumerate(STANDARD_COLORS):
            d = max(0, card.cost.get(c, 0) - self.bonuses[i])
            need.append(d)
            gold += d - min(self.tokens[i], d)
        return self.tokens[5] >= gold, need


@dataclass
class SplendorState:
    """Host snapshot of one device table (reference engine/state.py:74-87 field names)."""
    num_players: int
    bank: List[int]
    players: List[PlayerState]
    board: Dict[int, List[Optional[Card]]]
    decks: Dict[int, List[Card]]
    nobles: List[Optional[Noble]]
    to_play: int = 0
    turn_count: int = 1
    move_count: int = 0
    game_over: bool = False
    winner_index: Optional[int] = None
    turn_limit_reached: bool = False

    def copy(self) -> "SplendorState":
        """Independent lists, shared cards and nobles (state.py:89-104)."""
        return SplendorState(
            num_players=self.num_players, bank=list(self.bank),
            players=[PlayerState(tokens=list(p.tokens), bonuses=list(p.bonuses), prestige=p.prestige,
                                 reserved=list(p.reserved), revealed_reserved=list(p.revealed_reserved),
                                 nobles=list(p.nobles)) for p in self.players],
            board={t: list(v) for t, v in self.board.items()}, decks={t: list(v) for t, v in self.decks.items()},
            nobles=list(self.nobles), to_play=self.to_play, turn_count=self.turn_count, move_count=self.move_count,
            game_over=self.game_over, winner_index=self.winner_index, turn_limit_reached=self.turn_limit_reached)

    def cards(self):
        """Every Card object of this state (board, decks, reserved), by id."""
        out = {}
        for t in (1, 2, 3):
            for c in self.board[t]:
                if c is not None:
                    out[c.id] = c
            for c in self.decks[t]:
                out[c.id] = c
        for p in self.players:
            for c in p.reserved:
                out[c.id] = c
        return out

    def card_table(self):
        """int32 [90, 8] device card table with this state's edited cards, or None when every card of
        the state has its canonical data (then the shared device tables apply)."""
        base = canonical_card_rows()
        tbl = None
        for i, c in self.cards().items():
            row = card_row(c)
            if list(base[i]) != row:
                if tbl is None:
                    tbl = np.array(base, np.int32, copy=True)
                tbl[i] = row
        return tbl

    @classmethod
    def from_record(cls, r, cards=None):
        """numpy record of _native.TABLE_DTYPE -> SplendorState.  cards (optional, id -> Card): objects
        to reuse (a state derived from another keeps its Card objects, edits included); every other
        card is a fresh copy of the canonical data."""
        nobles = nobles_by_index()
        own = {} if cards is None else cards

        class _Cards:
            def __getitem__(self, i):
                c = own.get(i)
                if c is None:
                    c = own[i] = card_copy(i)
                return c
        cards = _Cards()
        P = int(r["num_players"])
        players = []
        for p in range(P):
            q = r["players"][p]
            n = int(q["n_reserved"])
            players.append(PlayerState(tokens=[int(x) for x in q["tokens"]], bonuses=[int(x) for x in q["bonuses"]],
                                       prestige=int(q["prestige"]),
                                       reserved=[cards[int(i)] for i in q["reserved"][:n]],
                                       revealed_reserved=[bool(x) for x in q["revealed"][:n]],
                                       nobles=[nobles[int(i)] for i in q["nobles"][:int(q["n_nobles"])]]))
        board = {t: [(cards[int(i)] if i >= 0 else None) for i in r["board"][(t - 1) * 4:t * 4]] for t in (1, 2, 3)}
        decks = {t: [cards[int(i)] for i in r["decks"][t - 1][:int(r["deck_len"][t - 1])]] for t in (1, 2, 3)}
        nob = [(nobles[int(i)] if i >= 0 else None) for i in r["nobles"][:int(r["n_nobles"])]]
        w = int(r["winner"])
        return cls(P, [int(x) for x in r["bank"]], players, board, decks, nob, int(r["to_play"]), int(r["turn_count"]),
                   int(r["move_count"]), bool(r["game_over"]), None if w < 0 else w, bool(r["turn_limit_reached"]))

    def to_record(self):
        from .._native import TABLE_DTYPE
        r = np.zeros((), TABLE_DTYPE)
        r["num_players"] = self.num_players
        r["bank"] = self.bank
        for p in range(4):
            q = r["players"][p]
            q["reserved"] = -1
            q["nobles"] = -1
            if p >= self.num_players:
                continue
            ps = self.players[p]
            q["tokens"], q["bonuses"], q["prestige"] = ps.tokens, ps.bonuses, ps.prestige
            n = len(ps.reserved)
            q["n_reserved"] = n
            q["reserved"][:n] = [c.id for c in ps.reserved]
            rev = list(ps.revealed_reserved) + [False] * n
            q["revealed"][:n] = [int(bool(x)) for x in rev[:n]]
            q["n_nobles"] = len(ps.nobles)
            q["nobles"][:len(ps.nobles)] = [nb.id - 1000 for nb in ps.nobles]
        r["board"] = [(c.id if c is not None else -1) for t in (1, 2, 3) for c in self.board[t]]
        r["decks"] = -1
        for t in (1, 2, 3):
            d = self.decks[t]
            r["deck_len"][t - 1] = len(d)
            r["decks"][t - 1][:len(d)] = [c.id for c in d]
        r["n_nobles"] = len(self.nobles)
        r["nobles"] = -1
        r["nobles"][:len(self.nobles)] = [(nb.id - 1000 if nb is not None else -1) for nb in self.nobles]
        r["to_play"], r["turn_count"], r["move_count"] = self.to_play, self.turn_count, self.move_count
        r["game_over"] = int(bool(self.game_over))
        r["winner"] = -1 if self.winner_index is None else self.winner_index
        r["turn_limit_reached"] = int(bool(self.turn_limit_reached))
        return r
