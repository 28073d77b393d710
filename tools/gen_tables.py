"""Derive the engine's constant tables from the reference's game data.

Reads the reference's card/noble JSON (human colour names, one object per
card) and writes ``splendor_gym/engine/data/tables.json`` in this project's
own compact, internal-colour-order format:

    cards:  [tier, bonus_colour, points, cost_w, cost_b, cost_g, cost_r, cost_k]
            one row per card id 0..89 (ids follow the reference's JSON order,
            reference engine/state.py:121-142)
    nobles: [req_w, req_b, req_g, req_r, req_k, points]
            one row per noble index 0..9 (reference id = 1000 + index,
            engine/state.py:160-174)

Colour map follows reference engine/state.py:16-23 (diamond→white,
sapphire→blue, emerald→green, ruby→red, onyx→black).

This is a one-off data-prep tool run in the build container; the output is
committed, so nothing at run time reads /root/reference.
"""
import json
import os
import sys

HUMAN = ["diamond", "sapphire", "emerald", "ruby", "onyx"]


def main(ref_root="/root/reference", out=None):
    data = os.path.join(ref_root, "splendor_gym", "engine", "data")
    with open(os.path.join(data, "cards.json")) as f:
        raw_cards = json.load(f)
    with open(os.path.join(data, "nobles.json")) as f:
        raw_nobles = json.load(f)
    cards = []
    for obj in raw_cards:
        cost = [int(obj.get("cost", {}).get(h, 0)) for h in HUMAN]
        cards.append([int(obj["tier"]), HUMAN.index(obj["bonus"]), int(obj.get("points", 0))] + cost)
    # tiers must be contiguous 40/30/20 (reference state.py:144-148)
    tiers = [c[0] for c in cards]
    assert tiers == [1] * 40 + [2] * 30 + [3] * 20, "unexpected card order"
    nobles = []
    for obj in raw_nobles:
        req = [int(obj.get("req", {}).get(h, 0)) for h in HUMAN]
        nobles.append(req + [int(obj.get("points", 3))])
    assert len(nobles) == 10
    out = out or os.path.join(os.path.dirname(__file__), "..", "splendor-gym_amd",
                              "splendor_gym", "engine", "data", "tables.json")
    with open(out, "w") as f:
        f.write('{"colour_order": ["white", "blue", "green", "red", "black"],\n')
        f.write(' "card_fields": ["tier", "bonus", "points", "cost_w", "cost_b", "cost_g", "cost_r", "cost_k"],\n')
        f.write(' "noble_fields": ["req_w", "req_b", "req_g", "req_r", "req_k", "points"],\n')
        f.write(' "cards": [\n')
        f.write(",\n".join("  " + json.dumps(c) for c in cards))
        f.write('\n ],\n "nobles": [\n')
        f.write(",\n".join("  " + json.dumps(n) for n in nobles))
        f.write("\n ]\n}\n")
    print("wrote", os.path.normpath(out))


if __name__ == "__main__":
    main(*sys.argv[1:])
