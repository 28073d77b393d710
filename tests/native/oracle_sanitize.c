/* Sanitizer driver for the CPU oracle (oracle/splendor_oracle.c), built by tests/test_host_cpu.py
 * with -fsanitize=address,undefined: deals for every player count, long uniform-random rollouts
 * with autoreset, env steps on crafted extremes (out-of-range and illegal actions, hundreds of
 * tokens to return, empty decks / boards, turn limit) — any out-of-bounds access, use of
 * uninitialised stack memory or signed overflow aborts the run.  Test infrastructure only. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/splendor_table.h"

typedef struct { uint32_t mt[624]; int index; } orc_mt_t;
void orc_set_tables(const int32_t *cards, const int32_t *nobles);
void orc_initial_state(spl_table_t *s, int P, uint32_t seed);
uint64_t orc_legal(const spl_table_t *s);
int orc_apply(spl_table_t *s, int a);
void orc_encode(const spl_table_t *s, int32_t *obs);
int orc_env_step(spl_table_t *s, int action, int32_t *obs, uint64_t *mask, float *reward, int32_t *terminated,
                 int32_t *flags, float *final_r, int32_t *has_final);
int64_t orc_random_rollout(int P, const uint64_t *pcg4, uint64_t policy_seed, int64_t n_steps, int64_t *episodes);

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(uint32_t n) {
    rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
    return (uint32_t)((rng >> 32) % n);
}

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    int32_t tables[90 * 8 + 10 * 6];
    FILE *f = fopen(argv[1], "rb");
    if (!f || fread(tables, sizeof(int32_t), 90 * 8 + 10 * 6, f) != 90 * 8 + 10 * 6) return 3;
    fclose(f);
    orc_set_tables(tables, tables + 90 * 8);
    int32_t obs[SPL_OBS_DIM];
    uint64_t mask;
    float r, fr[4];
    int32_t term, fl, hf;
    long checks = 0;
    for (int P = 2; P <= 4; ++P) {
        uint64_t pcg[4] = {0x1234567ull * P, 0x89abcdefull, 0x2468ull, 0x1357ull | 1ull};
        int64_t eps = 0;
        checks += orc_random_rollout(P, pcg, 99 + P, 20000, &eps);
        for (uint32_t seed = 0; seed < 300; ++seed) {
            spl_table_t s;
            orc_initial_state(&s, P, seed * 2654435761u);
            for (int step = 0; step < 400; ++step) {
                int a = (int)rnd(50) - 2;  /* out-of-range and illegal actions too */
                if (rnd(8) == 0) {         /* crafted extremes */
                    int p = s.to_play;
                    for (int c = 0; c < 6; ++c) s.players[p].tokens[c] = (int32_t)rnd(120);
                    if (rnd(4) == 0) s.deck_len[rnd(3)] = 0;
                    if (rnd(4) == 0) s.board[rnd(12)] = -1;
                    if (rnd(6) == 0) { s.move_count = 196 + (int32_t)rnd(4); s.turn_count = s.move_count / 2 + 1; }
                }
                int err = orc_env_step(&s, a, obs, &mask, &r, &term, &fl, fr, &hf);
                ++checks;
                if (err || term) orc_initial_state(&s, P, (uint32_t)rnd(1u << 31));
            }
        }
    }
    printf("OK %ld\n", checks);
    return 0;
}
