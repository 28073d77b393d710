// spl_rng.h — device RNGs for the Splendor engine (gfx950).
//
// * CPython MT19937 (random.Random(seed), Python 3.10 Modules/_randommodule.c) as a
//   REGISTER-ONLY stream: init_by_array is re-run as three sequential cursors instead of
//   materialising the 624-word state, so a lane needs ~20 VGPRs and no scratch.  Outputs
//   0..453 are produced in order (a deal needs <= 212 over 2e7 seeds).
// * numpy PCG64 + Generator.integers(0, 2**31-1): the per-table gymnasium np_random stream
//   that yields each episode's engine seed (reference envs/splendor_env.py:42-43).
// * Philox4x32-10 for the on-device uniform-random policy (no parity requirement: recorded
//   actions are replayed on the CPU oracle).
#pragma once
#include <stdint.h>
#ifndef SPL_HOST_UNIT_TEST
#include <hip/hip_runtime.h>
#endif

namespace spl {

// init_genrand(19650218): the fixed starting state of every init_by_array.
struct MTBase {
    uint32_t v[624];
    constexpr MTBase() : v() {
        v[0] = 19650218u;
        for (int i = 1; i < 624; ++i) v[i] = 1812433253u * (v[i - 1] ^ (v[i - 1] >> 30)) + (uint32_t)i;
    }
};
// Only three entries are ever needed directly (cursor start points); the rest is regenerated.
constexpr uint32_t kMTB0 = MTBase().v[0];
constexpr uint32_t kMTB1 = MTBase().v[1];
constexpr uint32_t kMTB396 = MTBase().v[396];

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

// one step of the twist: ((x & UPPER) | (y & LOWER)) >> 1 ^ mag01[y & 1]
__device__ __forceinline__ uint32_t mt_tw(uint32_t x, uint32_t y) {
    return ((((x & 0x80000000u) | (y & 0x7fffffffu)) >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u));
}

// init_genrand's recurrence: b_i from b_{i-1}.  Cursors regenerate the base table on the fly
// instead of loading it: b is wave-uniform, so it lives in SGPRs and runs on the scalar unit
// beside the vector chains (a scalar load per step would expose its latency every iteration).
__device__ __forceinline__ uint32_t mt_base_next(uint32_t b, int i) {
    return 1812433253u * (b ^ (b >> 30)) + (uint32_t)i;
}

// Cursor over the post-init_by_array state s[i], i >= 2, produced in increasing i.
//   loop 1:  a_i = (b_i ^ ((a_{i-1} ^ a_{i-1} >> 30) * 1664525)) + key[j] + j,  j = (i-1) % keylen
//   loop 2:  c_i = (a_i ^ ((c_{i-1} ^ c_{i-1} >> 30) * 1566083941)) - i        (= s_i, i >= 2)
struct MTCursor {
    uint32_t b, a, c;  // b = b_{i-1} (uniform), a = a_{i-1}, c = c_{i-1}
    __device__ __forceinline__ uint32_t step(int i, uint32_t add_even, uint32_t add_odd) {
        const uint32_t add = ((i - 1) & 1) ? add_odd : add_even;
        b = mt_base_next(b, i);
        a = (b ^ ((a ^ (a >> 30)) * 1664525u)) + add;
        c = (a ^ ((c ^ (c >> 30)) * 1566083941u)) - (uint32_t)i;
        return c;
    }
};

// Streaming CPython MT19937 for a seed < 2**64 (key length 1 or 2).  Usage: init(), then
// next(j) for j = 0, 1, 2, ... in order, with j UNIFORM across the active lanes (the base
// table is read with scalar loads).  Valid for j < kMaxOut.
struct MTStream {
    static constexpr int kMaxOut = 454;
    uint32_t add_even, add_odd;
    uint32_t a1, a1p, s1;        // a_1 (loop 1), a'_1 (loop 1's wrap iteration), final s_1
    uint32_t r_a0, r_c0;         // (a_396, c_396): restart point of the +397 / +170 cursor
    MTCursor L, R, M;            // s_{j+1};  s_{j+397} (phase A) / s_{j+170} (phase B);  s_{j-226}
    uint32_t sj, smj;            // s_j and s_{j-227}

    __device__ __forceinline__ void init(uint64_t seed) {
        const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
        const bool two = k1 != 0u;  // random_seed(): key length = max(1, ceil(bits / 32))
        add_even = k0;
        add_odd = two ? k1 + 1u : k0;
        // loop 1 to the end: a_623
        a1 = (kMTB1 ^ ((kMTB0 ^ (kMTB0 >> 30)) * 1664525u)) + k0;
        uint32_t a = a1, b = kMTB1;
#pragma unroll 8
        for (int i = 2; i < 624; ++i) {
            const uint32_t add = ((i - 1) & 1) ? add_odd : add_even;
            b = mt_base_next(b, i);
            a = (b ^ ((a ^ (a >> 30)) * 1664525u)) + add;
        }
        // 624th loop-1 iteration wraps to i = 1 with mt[0] = a_623, j = 623 % keylen
        a1p = (a1 ^ ((a ^ (a >> 30)) * 1664525u)) + (two ? k1 + 1u : k0);
        // loop 2 to the end: c_623, remembering (a_396, c_396)
        MTCursor cur{kMTB1, a1, a1p};
#pragma unroll 4
        for (int i = 2; i < 397; ++i) cur.step(i, add_even, add_odd);
        r_a0 = cur.a;  // (a_396, c_396)
        r_c0 = cur.c;
#pragma unroll 4
        for (int i = 397; i < 624; ++i) cur.step(i, add_even, add_odd);
        s1 = (a1p ^ ((cur.c ^ (cur.c >> 30)) * 1566083941u)) - 1u;
        L = MTCursor{kMTB1, a1, a1p};
        R = MTCursor{kMTB396, r_a0, r_c0};
        sj = 0x80000000u;  // s_0
    }

    // Output j (tempered).  j must advance 0, 1, 2, ... uniformly.
    __device__ __forceinline__ uint32_t next(int j) {
        const uint32_t sj1 = (j == 0) ? s1 : L.step(j + 1, add_even, add_odd);
        uint32_t y;
        if (j < 227) {
            y = R.step(j + 397, add_even, add_odd) ^ mt_tw(sj, sj1);
        } else {
            if (j == 227) {  // phase B: mt_new[j] = s_{j+170} ^ tw(s_{j-227}, s_{j-226}) ^ tw(s_j, s_{j+1})
                R = MTCursor{kMTB396, r_a0, r_c0};
                M = MTCursor{kMTB1, a1, a1p};
                smj = 0x80000000u;
            }
            const uint32_t smj1 = (j == 227) ? s1 : M.step(j - 226, add_even, add_odd);
            y = R.step(j + 170, add_even, add_odd) ^ mt_tw(smj, smj1) ^ mt_tw(sj, sj1);
            smj = smj1;
        }
        sj = sj1;
        return mt_temper(y);
    }
};

// One lane's full CPython MT19937 state (624 words) in a caller-provided LDS region: the
// continuation path of a lane that needs more outputs than MTStream streams (kMaxOut).  Run by ONE
// lane at a time (the caller loops over the lanes that need it), so the region is shared by the
// wave and no cross-lane operation is involved.  init() is a serial pass over the state; never
// taken by natural play: crafted states with hundreds of tokens to return.
struct LaneMT {
    uint32_t *m;  // >= 624 words of LDS owned by the calling lane for the duration
    int idx;

    // random.seed(seed) for 0 <= seed < 2^64: init_genrand(19650218), then init_by_array with a
    // key of 1 or 2 32-bit words (Modules/_randommodule.c)
    __device__ void init(uint64_t seed) {
        const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
        const int keylen = key[1] ? 2 : 1;
        m[0] = 19650218u;
        for (int i = 1; i < 624; ++i) m[i] = 1812433253u * (m[i - 1] ^ (m[i - 1] >> 30)) + (uint32_t)i;
        int i = 1, j = 0;
        for (int k = 624; k; --k) {
            m[i] = (m[i] ^ ((m[i - 1] ^ (m[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
            ++i;
            ++j;
            if (i >= 624) {
                m[0] = m[623];
                i = 1;
            }
            if (j >= keylen) j = 0;
        }
        for (int k = 623; k; --k) {
            m[i] = (m[i] ^ ((m[i - 1] ^ (m[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
            ++i;
            if (i >= 624) {
                m[0] = m[623];
                i = 1;
            }
        }
        m[0] = 0x80000000u;
        idx = 624;
    }

    __device__ void twist() {
        int k = 0;
        for (; k < 624 - 397; ++k) m[k] = m[k + 397] ^ mt_tw(m[k], m[k + 1]);
        for (; k < 623; ++k) m[k] = m[k - 227] ^ mt_tw(m[k], m[k + 1]);
        m[623] = m[396] ^ mt_tw(m[623], m[0]);
        idx = 0;
    }

    // continue the stream at output `j` (< 624) of the first block
    __device__ void start_at(int j) {
        twist();
        idx = j;
    }

    __device__ uint32_t next() {
        if (idx >= 624) twist();
        return mt_temper(m[idx++]);
    }
};

__device__ __forceinline__ int bit_length(uint32_t n) { return n ? 32 - __clz((int)n) : 0; }

// ---- numpy PCG64 ------------------------------------------------------------------------
struct Pcg64 {
    uint64_t s_hi, s_lo, inc_hi, inc_lo;
    uint32_t has32, u32;

    __device__ __forceinline__ uint64_t next64() {
        typedef unsigned __int128 u128;
        const u128 mul = ((u128)2549297995355413924ULL << 64) | 4865540595714422341ULL;
        u128 s = ((u128)s_hi << 64) | s_lo;
        s = s * mul + (((u128)inc_hi << 64) | inc_lo);
        s_hi = (uint64_t)(s >> 64);
        s_lo = (uint64_t)s;
        const uint64_t x = s_hi ^ s_lo;
        const unsigned rot = (unsigned)(s_hi >> 58);
        return (x >> rot) | (x << ((64u - rot) & 63u));
    }
    __device__ __forceinline__ uint32_t next32() {
        if (has32) {
            has32 = 0;
            return u32;
        }
        const uint64_t n = next64();
        has32 = 1;
        u32 = (uint32_t)(n >> 32);
        return (uint32_t)n;
    }
    // numpy's stream increment is (initseq << 1) | 1: an even one is an unseeded (zeroed) record
    __device__ __forceinline__ bool valid() const { return (inc_lo & 1u) != 0; }

    // Generator.integers(0, 2**31 - 1) -> buffered_bounded_lemire_uint32(rng = 2**31 - 2).
    // A draw is rejected with probability 2 / 2**32, so the retry bound (never reached by a
    // seeded stream: 2**-992) only keeps an invalid record from spinning forever.
    __device__ __forceinline__ uint32_t engine_seed() {
        const uint32_t rng_excl = 2147483647u;
        uint64_t m = (uint64_t)next32() * rng_excl;
        uint32_t left = (uint32_t)m;
        if (left < rng_excl) {
            const uint32_t threshold = (0xFFFFFFFFu - 2147483646u) % rng_excl;
            for (int tries = 0; left < threshold && tries < 32; ++tries) {
                m = (uint64_t)next32() * rng_excl;
                left = (uint32_t)m;
            }
        }
        return (uint32_t)(m >> 32);
    }
};

// ---- Philox4x32-10 -------------------------------------------------------------------------
__device__ __forceinline__ uint4 philox4x32(uint4 ctr, uint2 key) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, ctr.x), lo0 = 0xD2511F53u * ctr.x;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, ctr.z), lo1 = 0xCD9E8D57u * ctr.z;
        ctr = make_uint4(hi1 ^ ctr.y ^ key.x, lo1, hi0 ^ ctr.w ^ key.y, lo0);
        key.x += 0x9E3779B9u;
        key.y += 0xBB67AE85u;
    }
    return ctr;
}

}  // namespace spl
