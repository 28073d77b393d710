// spl_layout.h — HBM layout of a Splendor arena and the packed per-table state words.
//
// One wavefront lane owns one table.  The mutable table state lives in 32-bit WORD PLANES:
// plane w holds word w of every table, so lane t touching word w reads plane[w * n + t] and a
// wave moves 256 contiguous bytes per plane (coalesced).  Words (bytes little-endian):
//
//   SW_BANK0   bank white, blue, green, red
//   SW_BANK1   bank black, gold, to_play, turn_count
//   SW_MISC    move_count (16) | status (8) | winner+1 (8)
//   SW_BOARD+t board tier t+1, slots 0..3 (card id, 0xFF = empty)
//   SW_DECK    deck_len tier 1..3, number of visible noble slots
//   SW_NOB0    noble index in visible slots 0..3 (0xFF = none)
//   SW_NOB1    slot 4 index | slot owners << 8 (3 bits per slot: 0 visible, p+1 taken by
//              player p, 7 taken by an unknown player)
//   PW(p,0..3) player p: tokens w b g r | tokens k, gold, bonus w, b | bonus g, r, k, prestige |
//              n_reserved (bits 0-1) + revealed (bits 2-4), reserved card ids 0..2 (0xFF none)
//
// The 13 observation bytes of a player (tokens 6, bonuses 5, prestige, n_reserved —
// reference engine/encode.py:131-142) are exactly PW0, PW1, PW2 and (PW3 & 3).
//
// Deck storage: kSlotRecords 128-byte SLOT RECORDS per table (AoS, [n][4][128]), used as a
// ring.  The live record (status bits ST_ACTIVE) holds the table's deck (bytes 0..89: tier 1 at
// 0, tier 2 at 40, tier 3 at 70, list order, top = deck_len-1); the next records in ring order
// are the POOL: the next episodes' deals, prepared ahead from the table's engine-seed stream by
// the refill kernel.  ST_PEND counts pool records consumed and not yet re-dealt (0..3; the LAST
// `pend` records in ring order are the free ones).  Record bytes 96..115 hold the deal's board
// and noble words, 124..127 its engine seed (diagnostic).  The next pool's board and noble
// words are also kept in their own word planes (PL_*), read with the state at the top of every
// step, so a same-step autoreset needs no late gather.
#pragma once
#include <stdint.h>

namespace spl {

enum : int {
    SW_BANK0 = 0,
    SW_BANK1 = 1,
    SW_MISC = 2,
    SW_BOARD = 3,
    SW_DECK = 6,
    SW_NOB0 = 7,
    SW_NOB1 = 8,
    SW_COUNT = 9,
};
__host__ __device__ constexpr int num_words(int P) { return SW_COUNT + 4 * P; }
__host__ __device__ constexpr int pw_index(int p, int k) { return SW_COUNT + 4 * p + k; }

// SW_MISC status bits
constexpr uint32_t ST_GAME_OVER = 1u << 16;
constexpr uint32_t ST_TURN_LIMIT = 1u << 17;
constexpr int ST_ACTIVE_SHIFT = 18;        // 2 bits: slot record (0..2) holding the live deck
constexpr uint32_t ST_ACTIVE = 3u << ST_ACTIVE_SHIFT;
constexpr int ST_PEND_SHIFT = 20;          // 2 bits: pool records consumed, not yet re-dealt
constexpr uint32_t ST_PEND = 3u << ST_PEND_SHIFT;
constexpr int kSlotRecords = 4;            // live record + up to 3 pool deals (ST_PEND <= 3)

constexpr int kSlotBytes = 128;
constexpr int kRecTail = 96;    // board x3, nob0, nob1 words of the deal
constexpr int kRecSeed = 124;   // engine seed of the deal (diagnostic)

// pool planes: the pool deal's SW_BOARD.. and SW_NOB0/1 words (SW_DECK at deal is a constant)
enum : int { PL_BOARD = 0, PL_NOB0 = 3, PL_NOB1 = 4, PL_COUNT = 5 };
constexpr int kPcgBytes = 64;   // per-table numpy PCG64 record: s_hi s_lo inc_hi inc_lo has32 u32

__host__ __device__ constexpr int tier_base(int t) { return t == 0 ? 0 : (t == 1 ? 40 : 70); }
__host__ __device__ constexpr int tier_size(int t) { return t == 0 ? 40 : (t == 1 ? 30 : 20); }

// token-return RNG table domain (engine/rules.py:170-175 seed fields):
//   turn_count < 128, to_play < 4, sum(tokens) in 11..13, sum(bank) < 16
constexpr int kLutTc = 128, kLutTp = 4, kLutSt = 3, kLutSb = 16;
constexpr int kLutEntries = kLutTc * kLutTp * kLutSt * kLutSb;
constexpr int kLutOutputs = 40;  // top 3 bits of the first 40 MT outputs, 10 per word

// Rollout-store delegation (k_rollout_store_<P>p at 64 tables per workgroup with per-step outputs; see
// the kernel): per pair of workgroups (2q, 2q+1), kDelegTasks staged steps (the odd workgroup's
// 64 tables' state words after the step, [word][lane] u32, room for 4 players) and the flags, one
// 128-byte line each: the two workgroups' launch counters, then ready and taken per task.
constexpr int kDelegTasks = 24;  // every 6th step of a 128-step launch (ppo_splendor.py --num-steps 128)
constexpr int kDelegPayload = 64 * 4 * num_words(4);  // 6 400 B
constexpr int kFlagLine = 32;            // u32 words per flag
enum : int { DF_PROD_EPOCH = 0, DF_CONS_EPOCH = 1, DF_TASKS = 2 };  // + 2 * task + {0 ready, 1 taken}
constexpr int kDelegFlagWords = (DF_TASKS + 2 * kDelegTasks) * kFlagLine;

// Partner hand-off of the six-wave dealer rollout (k_rollout_store_dealer2_*; see the kernel): team j of
// workgroups 2q and 2q+1 (XCCs x and x^1) share pair (q*2 + j) of the same arena lines and slots.  Side s
// (0: workgroup 2q) posts into task slots [s*kPartnerSlots, (s+1)*kPartnerSlots); its launch counter is
// line DF_PROD_EPOCH + s, its progress and done words the taken lines of its first two slots.
constexpr int kPartnerSlots = 12;
static_assert(2 * kPartnerSlots <= kDelegTasks, "both sides' partner slots fit the delegation slots");
__host__ __device__ constexpr int pt_ready_line(int slot) { return DF_TASKS + 2 * slot; }
__host__ __device__ constexpr int pt_progress_line(int side) { return DF_TASKS + 2 * (side * kPartnerSlots) + 1; }
__host__ __device__ constexpr int pt_done_line(int side) { return DF_TASKS + 2 * (side * kPartnerSlots + 1) + 1; }
__host__ __device__ constexpr int pt_epoch_line(int side) { return DF_PROD_EPOCH + side; }

// Legal-mask cache (ABI 9): [2][n] u32, legal_moves of the table's STORED state as written by the
// kernel that stored it — word 0 mask bits 0..31, word 1 bits 32..44 | card-table tag << 16.  A reader
// trusts it only when the tag equals its context's nonzero tag (one tag per distinct card table in the
// process: contexts of equal tables share it, an edited table gets its own), and every kernel that
// stores table state writes the mask it computed or tag 0 (unknown).  spl_step reads it so its pre-step
// check needs no legal_moves evaluation.
constexpr uint32_t kLegalHiBits = 0x1FFFu;
constexpr int kLegalTagShift = 16;
constexpr uint32_t kLegalTagMax = 0xFFFFu;  // tags 1..65535 (16 bits above the mask's 13)

struct ArenaLayout {
    int64_t planes, pool, slots, pcg, deleg, dflags, legal, total;
};

__host__ __device__ inline int64_t align256(int64_t x) { return (x + 255) & ~int64_t(255); }

__host__ __device__ inline ArenaLayout arena_layout(int64_t n, int P) {
    ArenaLayout L;
    L.planes = 0;
    L.pool = align256(L.planes + (int64_t)num_words(P) * n * 4);
    L.slots = align256(L.pool + (int64_t)PL_COUNT * n * 4);
    L.pcg = align256(L.slots + n * kSlotRecords * kSlotBytes);
    L.deleg = align256(L.pcg + n * kPcgBytes);
    L.dflags = align256(L.deleg + (n / 128) * kDelegTasks * (int64_t)kDelegPayload);
    L.legal = align256(L.dflags + (n / 128) * kDelegFlagWords * 4);
    L.total = align256(L.legal + 2 * n * 4);
    return L;
}

}  // namespace spl
