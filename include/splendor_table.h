/*
 * splendor_table.h — host view of ONE Splendor table (plain C, no HIP types).
 *
 * This record is the exchange format between the device arena (spl_table_download /
 * spl_table_upload in splendor_amd.h), the CPU oracle (oracle/splendor_oracle.c) and the
 * Python host view.  It restates the reference's mutable state objects with plain int32:
 *
 *   reference SplendorState   splendor_gym/engine/state.py:74-87
 *   reference PlayerState     splendor_gym/engine/state.py:52-59
 *
 * Encodings: card id 0..89 = position in the reference's cards.json (tier 1 = 0..39,
 * tier 2 = 40..69, tier 3 = 70..89; engine/state.py:121-142); noble index 0..9 = reference
 * noble id − 1000 (engine/state.py:161-174); −1 = empty board slot / taken noble /
 * unused list entry / `winner_index is None`.  Colours use the reference's internal order
 * white, blue, green, red, black, gold (engine/state.py:10).
 */
#ifndef SPLENDOR_TABLE_H
#define SPLENDOR_TABLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPL_MAX_PLAYERS 4
#define SPL_NUM_CARDS 90
#define SPL_NUM_NOBLES 10
#define SPL_OBS_DIM 297      /* engine/encode.py:74 */
#define SPL_NUM_ACTIONS 45   /* engine/encode.py:32 */

typedef struct spl_player_s {
    int32_t tokens[6];       /* PlayerState.tokens */
    int32_t bonuses[5];      /* PlayerState.bonuses */
    int32_t prestige;        /* PlayerState.prestige */
    int32_t n_reserved;      /* len(PlayerState.reserved), 0..3 */
    int32_t reserved[3];     /* card ids, in list order */
    int32_t revealed[3];     /* PlayerState.revealed_reserved */
    int32_t n_nobles;        /* len(PlayerState.nobles) */
    int32_t nobles[5];       /* noble indices */
} spl_player_t;

typedef struct spl_table_s {
    int32_t num_players;     /* 2..4 */
    int32_t bank[6];
    spl_player_t players[SPL_MAX_PLAYERS];
    int32_t board[12];       /* tier-major, slot-minor (engine/encode.py:46-47) */
    int32_t deck_len[3];
    int32_t decks[3][40];    /* deck order as in the reference list: top of deck = deck_len-1 */
    int32_t n_nobles;        /* visible noble slots = min(P+1, 10) (engine/state.py:194) */
    int32_t nobles[5];       /* noble index per visible slot, −1 once taken */
    int32_t to_play;
    int32_t turn_count;
    int32_t move_count;
    int32_t game_over;
    int32_t winner;          /* −1 = None */
    int32_t turn_limit_reached;
} spl_table_t;

#ifdef __cplusplus
}
#endif
#endif /* SPLENDOR_TABLE_H */
