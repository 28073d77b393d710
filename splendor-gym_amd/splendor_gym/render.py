"""Text rendering of a host state snapshot (the reference renders through
scripts/game_logger.py:159-220 format_game_state; this is a compact equivalent)."""
from .engine.state import STANDARD_COLORS, TOKEN_COLORS

_ABBR = {"white": "W", "blue": "U", "green": "G", "red": "R", "black": "K", "gold": "*"}


def _card(c):
    if c is None:
        return "[ -- ]"
    cost = "".join(f"{v}{_ABBR[k]}" for k, v in c.cost.items())
    return f"[#{c.id} T{c.tier} {_ABBR[c.color]} {c.points}p {cost}]"


def format_game_state(s):
    if s is None:
        return "<no state: call reset()>"
    lines = [f"Turn {s.turn_count} (move {s.move_count}) | to play: P{s.to_play}"
             + (" | GAME OVER" if s.game_over else "") + (" | TURN LIMIT" if s.turn_limit_reached else "")
             + ("" if s.winner_index is None else f" | winner P{s.winner_index}")]
    lines.append("Bank: " + " ".join(f"{_ABBR[c]}{n}" for c, n in zip(TOKEN_COLORS, s.bank)))
    nob = ["--" if n is None else f"N{n.id}:" + "".join(f"{v}{_ABBR[k]}" for k, v in n.requirements.items())
           for n in s.nobles]
    lines.append("Nobles: " + " ".join(nob))
    for t in (3, 2, 1):
        lines.append(f"Tier {t} ({len(s.decks[t])} left): " + " ".join(_card(c) for c in s.board[t]))
    for i, p in enumerate(s.players):
        toks = " ".join(f"{_ABBR[c]}{n}" for c, n in zip(TOKEN_COLORS, p.tokens))
        bon = " ".join(f"{_ABBR[c]}{n}" for c, n in zip(STANDARD_COLORS, p.bonuses))
        res = " ".join((_card(c) if r else "[hidden " + _card(c) + "]") for c, r in zip(p.reserved, p.revealed_reserved))
        lines.append(f"P{i}{'*' if i == s.to_play else ' '} prestige {p.prestige} | tokens {toks} | bonuses {bon}"
                     f" | nobles {len(p.nobles)} | reserved {res or '-'}")
    return "\n".join(lines)
