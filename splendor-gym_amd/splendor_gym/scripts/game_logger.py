"""Human-readable game text: the reference's compact logger (splendor_gym/scripts/game_logger.py:48-288),
which SplendorEnv.render prints (envs/splendor_env.py:119-126).

Same public surface and byte-identical text (pinned by tests/golden/render.json, generated from the
reference): SplendorGameLogger.format_game_state / decode_action / get_legal_actions_description /
log_game_step / print_game_log, GameLog, run_logged_game, and the CLI.  Works on any object with the
reference SplendorState fields (this package's host view included).

Notation: colour letters w b g r k and G for gold; a card is "<colour>-<points>pt-<cost>" with the
cost in white..black order ("free" if none); a noble "<points>pt-<requirements>".
"""
import argparse
import random
from dataclasses import dataclass
from typing import Dict, List, Optional

from ..engine.encode import (BUY_RESERVED_OFFSET, BUY_VISIBLE_OFFSET, RESERVE_BLIND_OFFSET, RESERVE_VISIBLE_OFFSET,
                             TAKE2_OFFSET, TAKE3_COMBOS, TOTAL_ACTIONS)
from ..engine.state import STANDARD_COLORS, TOKEN_COLORS

LETTER = dict(zip(TOKEN_COLORS, "wbgrkG"))


def _amounts(pairs, empty):
    """'<n><letter>' for every positive amount, in the given colour order."""
    s = "".join(f"{n}{LETTER[c]}" for c, n in pairs if n > 0)
    return s or empty


def card_text(card) -> str:
    if not card:
        return "[empty]"
    cost = _amounts(((c, card.cost.get(c, 0)) for c in STANDARD_COLORS), "free")
    return f"{LETTER[card.color]}-{card.points}pt-{cost}"


def noble_text(noble) -> str:
    req = _amounts(((c, noble.requirements.get(c, 0)) for c in STANDARD_COLORS), "") if noble.requirements else "free"
    return f"{noble.points}pt-{req}"


def _slot(action, base):
    k = action - base
    return 1 + k // 4, k % 4


@dataclass
class GameLog:
    turn: int
    player: int
    state_before: str
    action: str
    state_after: str
    legal_actions: List[str]


class SplendorGameLogger:
    """Compact text of states and actions; collects GameLog records of a played game."""

    def __init__(self):
        self.logs: List[GameLog] = []
        self.color_abbrev: Dict[str, str] = dict(LETTER)
        self.abbrev_to_color = {v: k for k, v in LETTER.items()}

    # ---- actions -----------------------------------------------------------------------
    def decode_action(self, action: int, state) -> str:
        a = int(action)
        if a < 0 or a >= TOTAL_ACTIONS:
            return f"Action{a}"
        if a < TAKE2_OFFSET:
            # take-3 follows the reduced rule: the colours actually taken depend on the bank
            avail = [c for c in range(5) if state.bank[c] >= 1]
            if len(avail) >= 3:
                return "Take3: " + "".join(LETTER[STANDARD_COLORS[c]] for c in TAKE3_COMBOS[a])
            if len(avail) == 2:
                return "Take2: " + "".join(LETTER[STANDARD_COLORS[c]] for c in avail) + " (reduced)"
            if len(avail) == 1:
                return f"Take1: {LETTER[STANDARD_COLORS[avail[0]]]} (reduced)"
            return f"Action{a}"
        if a < BUY_VISIBLE_OFFSET:
            ch = LETTER[STANDARD_COLORS[a - TAKE2_OFFSET]]
            return f"Take2: {ch}{ch}"
        if a < RESERVE_BLIND_OFFSET:
            verb, base = ("Buy", BUY_VISIBLE_OFFSET) if a < RESERVE_VISIBLE_OFFSET else ("Reserve", RESERVE_VISIBLE_OFFSET)
            tier, slot = _slot(a, base)
            return f"{verb}: T{tier}S{slot + 1} {card_text(state.board[tier][slot])}"
        if a < BUY_RESERVED_OFFSET:
            return f"Reserve: T{a - RESERVE_BLIND_OFFSET + 1} blind"
        k = a - BUY_RESERVED_OFFSET
        held = state.players[state.to_play].reserved
        return f"BuyReserved: #{k + 1} {card_text(held[k]) if k < len(held) else '[empty]'}"

    # ---- states ------------------------------------------------------------------------
    def _player_line(self, i, p, to_play) -> str:
        toks = _amounts(zip(TOKEN_COLORS, p.tokens), "none")
        bonus = _amounts(zip(STANDARD_COLORS, p.bonuses), "none")
        res = ", ".join(card_text(c) for c in p.reserved) or "none"
        nob = ", ".join(noble_text(n) for n in p.nobles) or "none"
        mark = ">>>" if i == to_play else "   "
        return f"{mark} P{i}: {toks} | bonus:{bonus} | pts:{p.prestige} | reserved:[{res}] | nobles:[{nob}]"

    def format_game_state(self, state, player_perspective: int = -1) -> str:
        moves = f"M{state.move_count}" if hasattr(state, "move_count") else ""
        out = [f"=== TURN {state.turn_count}{moves} - P{state.to_play} to move ===",
               "Bank: " + _amounts(zip(TOKEN_COLORS, state.bank), "none")]
        out += [self._player_line(i, p, state.to_play) for i, p in enumerate(state.players)]
        out.append("Board:")
        out += [f"  T{t}: " + " | ".join(card_text(state.board[t][s]) for s in range(4)) for t in (3, 2, 1)]
        shown = [noble_text(n) for n in state.nobles if n is not None]
        out.append("Nobles: " + (" | ".join(shown) if shown else "none"))
        out.append("Decks: " + " ".join(f"T{t}:{len(state.decks[t])}" for t in (1, 2, 3)))
        return "\n".join(out)

    def get_legal_actions_description(self, state) -> List[str]:
        from ..engine import legal_moves  # device-evaluated rules (engine/rules.py)
        return [f"{a}: {self.decode_action(a, state)}" for a, ok in enumerate(legal_moves(state)) if ok]

    # ---- logs --------------------------------------------------------------------------
    def log_game_step(self, state_before, action: int, state_after):
        self.logs.append(GameLog(turn=state_before.turn_count, player=state_before.to_play,
                                 state_before=self.format_game_state(state_before),
                                 action=self.decode_action(action, state_before),
                                 state_after=self.format_game_state(state_after),
                                 legal_actions=self.get_legal_actions_description(state_before)))

    def print_game_log(self, show_legal_actions: bool = False, max_turns: Optional[int] = None):
        rule = "=" * 80
        print("\n" + rule + "\nSPLENDOR GAME LOG (Full Rounds)\n" + rule)
        by_turn: Dict[int, List[GameLog]] = {}
        for log in self.logs:
            by_turn.setdefault(log.turn, []).append(log)
        for shown, turn in enumerate(sorted(by_turn), start=1):
            if max_turns and shown > max_turns:
                print(f"\n... (showing first {max_turns} full turns only) ...")
                break
            group = by_turn[turn]
            print(f"\n{'=' * 20} TURN {turn} {'=' * 20}")
            for half, log in enumerate(group):
                print(f"\n--- {'FIRST HALF' if half == 0 else 'SECOND HALF'} (Player {log.player}) ---")
                print(log.state_before)
                if show_legal_actions:
                    print("Legal actions:")
                    for d in log.legal_actions[:10]:
                        print(f"  {d}")
                    if len(log.legal_actions) > 10:
                        print(f"  ... ({len(log.legal_actions) - 10} more)")
                    print("")
                print(f"P{log.player} ACTION: {log.action}")
                print("")
            print("--- TURN END STATE ---")
            print(group[-1].state_after)
            print("\n" + "-" * 60 + "\n")


def format_game_state(state) -> str:
    """Module-level shorthand of SplendorGameLogger().format_game_state."""
    return SplendorGameLogger().format_game_state(state)


def run_logged_game(policy_type: str = "random", seed: int = 42, max_turns: Optional[int] = None) -> SplendorGameLogger:
    """One logged game on the GPU-backed SplendorEnv (scripts/game_logger.py:291-367): random
    (random.Random(seed + 1000)), first-legal or interactive action choice."""
    from ..engine import winner
    from ..envs import SplendorEnv
    env = SplendorEnv(num_players=2)
    logger = SplendorGameLogger()
    obs, info = env.reset(seed=seed)
    rng = random.Random(seed + 1000)
    for step in range(1000):
        if max_turns and step >= 2 * max_turns:
            break
        before = env.state.copy()
        legal = [a for a, ok in enumerate(info["action_mask"]) if ok]
        if not legal:
            print("No legal actions available - game should have ended!")
            break
        if policy_type == "random":
            action = rng.choice(legal)
        elif policy_type == "first":
            action = legal[0]
        else:
            action = _ask(logger, before, legal)
        obs, reward, terminated, truncated, info = env.step(action)
        after = env.state.copy()
        logger.log_game_step(before, action, after)
        if terminated or truncated:
            print(f"\nGAME ENDED after {step + 1} steps!")
            if terminated:
                w = winner(after)
                print(f"Winner: Player {w}" if w is not None else "Game ended in a draw")
            break
    return logger


def _ask(logger, state, legal):
    print(logger.format_game_state(state))
    print("\nLegal actions:")
    for i, a in enumerate(legal):
        print(f"{i}: {logger.decode_action(a, state)}")
    while True:
        try:
            k = int(input("Choose action index (0-based): "))
        except (ValueError, KeyboardInterrupt):
            print("Invalid input, try again.")
            continue
        if 0 <= k < len(legal):
            return legal[k]
        print("Invalid choice, try again.")


def main():
    ap = argparse.ArgumentParser(description="Run and log Splendor games for verification")
    ap.add_argument("--policy", type=str, default="random", choices=["random", "first", "interactive"])
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--show-legal", action="store_true")
    ap.add_argument("--max-turns", type=int)
    ap.add_argument("--output", type=str)
    args = ap.parse_args()
    print(f"Running Splendor game with {args.policy} policy (seed: {args.seed})")
    logger = run_logged_game(args.policy, args.seed, args.max_turns)
    if args.output:
        import contextlib
        with open(args.output, "w") as f, contextlib.redirect_stdout(f):
            logger.print_game_log(args.show_legal, args.max_turns)
        print(f"Game log saved to {args.output}")
    else:
        logger.print_game_log(args.show_legal, args.max_turns)


if __name__ == "__main__":
    main()
