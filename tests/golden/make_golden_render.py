"""Fixtures for the host view / render surface: the REFERENCE scripts/game_logger.py
SplendorGameLogger (format_game_state, decode_action, get_legal_actions_description) on a set of
states, and SplendorEnv.render() text after seeded resets + scripted plies.  Loaded as in
make_golden.py (stub parent package + gymnasium stand-in).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_render.py     # here, with /root/reference

Writes tests/golden/render.json:
  states: [{name, view, text, actions: [decode_action(a) for a in 0..44], legal: [...]}]
  env:    [{seed, actions, text}]   (env.reset(seed) then `actions`, then env.render())
"""
import contextlib
import io
import json
import os
import random

import make_golden as mg  # noqa: F401  (installs the reference + gymnasium stand-in)
from schema import from_ref_state

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    from splendor_gym.scripts.game_logger import SplendorGameLogger
    eng, st = mg.eng, mg.st
    lg = SplendorGameLogger()
    states = []

    def add(name, s):
        legal = eng.legal_moves(s)
        states.append(dict(name=name, view=from_ref_state(s), text=lg.format_game_state(s),
                           actions=[lg.decode_action(a, s) for a in range(45)],
                           legal=lg.get_legal_actions_description(s), mask=[int(x) for x in legal]))

    for P in (2, 3, 4):
        for seed in (0, 1, 42):
            add(f"initial_p{P}_{seed}", eng.initial_state(P, seed))
    # random legal play (python random, seeded): snapshots along the way, incl. terminal states
    for P, games in ((2, 12), (3, 3), (4, 3)):
        for g in range(games):
            rs = random.Random(1000 * P + g)
            s = eng.initial_state(P, 7000 + 31 * g + P)
            ply = 0
            while True:
                m = eng.legal_moves(s)
                legal = [i for i, x in enumerate(m) if x]
                if not legal or eng.is_terminal(s) or ply > 400:
                    break
                s = eng.apply_action(s, rs.choice(legal))
                ply += 1
                if ply % 9 == 0 or eng.is_terminal(s):
                    add(f"play_p{P}_g{g}_ply{ply}", s)
    # crafted: the reference tests' mutations (tests/test_draw_rule.py, test_take_reduced_colors.py)
    s = eng.initial_state(2, 123)
    s.bank[:] = [0, 0, 0, 0, 0, 0]
    s.bank[0], s.bank[2] = 1, 2
    add("reduced_two_colours", s)
    s = eng.initial_state(2, 123)
    s.bank[:] = [0, 0, 0, 3 - 3, 3, 0]
    add("reduced_one_colour", s)
    s = eng.initial_state(2, 0)
    s.bank[:] = [0] * 6
    p = s.players[s.to_play]
    p.tokens[:] = [10, 0, 0, 0, 0, 0]
    p.reserved = s.decks[1][:3]
    for t in (1, 2, 3):
        s.board[t] = [None, None, None, None]
    add("draw_no_legal", s)

    env_cases = []
    for seed in (0, 5, 123, 2024):
        env = mg.envmod.SplendorEnv(num_players=2)
        obs, info = env.reset(seed=seed)
        rs = random.Random(seed)
        acts = []
        for k in range(rs.choice([0, 3, 17, 40])):
            legal = [i for i, x in enumerate(info["action_mask"]) if x]
            if not legal:
                break
            a = rs.choice(legal)
            obs, r, term, trunc, info = env.step(a)
            acts.append(a)
            if term:
                break
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            env.render()
        env_cases.append(dict(seed=seed, actions=acts, text=buf.getvalue()))

    with open(os.path.join(HERE, "render.json"), "w") as f:
        json.dump(dict(states=states, env=env_cases), f, indent=0)
    print(len(states), "states,", len(env_cases), "env cases")


if __name__ == "__main__":
    main()
