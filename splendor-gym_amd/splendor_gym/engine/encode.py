"""Action and observation layout (reference splendor_gym/engine/encode.py:12-74).

The same names and values as the reference so ``from splendor_gym.engine.encode import
OBSERVATION_DIM, TOTAL_ACTIONS`` (ppo_splendor.py:10) keeps working.  The encoding itself runs
on the GPU (splendor-gym_amd/csrc/spl_engine.hip, encode_row).

Observation (int32[297]):
    0-5     bank (white, blue, green, red, black, gold)
    6-18    current player: tokens 6, bonuses 5, prestige, #reserved
    19-31   next player (the "opponent"), same fields
    32-187  board 12 x [present, tier, points, colour one-hot 5, cost 5]  (tier-major)
    188-229 own reserved 3 x [card 13, revealed=1]
    230-271 opponent reserved 3 x [card 13, 1] if revealed, else zeros
    272-289 nobles[:3] x [present, requirement 5]
    290-292 deck sizes, 293 turn_count, 294 to_play, 295 move_count, 296 game_over and to_play==0
"""
from itertools import combinations

TAKE3_OFFSET = 0
TAKE3_COUNT = 10
TAKE2_OFFSET = TAKE3_OFFSET + TAKE3_COUNT
TAKE2_COUNT = 5
BUY_VISIBLE_OFFSET = TAKE2_OFFSET + TAKE2_COUNT
BUY_VISIBLE_COUNT = 12
RESERVE_VISIBLE_OFFSET = BUY_VISIBLE_OFFSET + BUY_VISIBLE_COUNT
RESERVE_VISIBLE_COUNT = 12
RESERVE_BLIND_OFFSET = RESERVE_VISIBLE_OFFSET + RESERVE_VISIBLE_COUNT
RESERVE_BLIND_COUNT = 3
BUY_RESERVED_OFFSET = RESERVE_BLIND_OFFSET + RESERVE_BLIND_COUNT
BUY_RESERVED_COUNT = 3
TOTAL_ACTIONS = BUY_RESERVED_OFFSET + BUY_RESERVED_COUNT

TAKE3_COMBOS = list(combinations(range(5), 3))

OBSERVATION_DIM = 297

OBS_BANK = slice(0, 6)
OBS_CURRENT = slice(6, 19)
OBS_OPPONENT = slice(19, 32)
OBS_BOARD = slice(32, 188)
OBS_RESERVED = slice(188, 272)
OBS_NOBLES = slice(272, 290)
OBS_DECKS = slice(290, 293)
OBS_TURN, OBS_TO_PLAY, OBS_MOVES, OBS_ROUND_OVER = 293, 294, 295, 296


def encode_take3_index(combo_index):
    return TAKE3_OFFSET + combo_index


def encode_take2_index(color_index):
    return TAKE2_OFFSET + color_index


def encode_buy_visible_index(tier, slot):
    return BUY_VISIBLE_OFFSET + (tier - 1) * 4 + slot


def encode_reserve_visible_index(tier, slot):
    return RESERVE_VISIBLE_OFFSET + (tier - 1) * 4 + slot


def encode_reserve_blind_index(tier):
    return RESERVE_BLIND_OFFSET + (tier - 1)


def encode_buy_reserved_index(slot):
    return BUY_RESERVED_OFFSET + slot


def encode_observation(state):
    """encode.py:124-187 for a host view, evaluated on the GPU (engine.rules.encode_observation)."""
    from .rules import encode_observation as _enc
    return _enc(state)
