// rt_mt.h -- numpy's legacy `np.random.rand` stream (MT19937) generated in parallel segments.
//
// Parity mode of Scene.render draws the primary-ray jitter from numpy's global RandomState in the
// reference's order (camera.py:51-85, utils/random.py:6-9, scene.py:78,81).  numpy's legacy
// generator (randomkit/mtrand, frozen by NEP 19; numpy 2.2.6 here) is MT19937: a window of 624
// 32-bit words x_j..x_{j+623} plus a position; every output is temper(x_k) of the next word, the
// window regenerating as x_{k+624} = x_{k+397} ^ twist(x_k, x_{k+1}); a double is
// ((w0 >> 5) * 2^26 + (w1 >> 6)) / 2^53 of two consecutive outputs.
//
// The word stream is cut into segments of L = 2^19 words.  Segment s starts from the window
// W_{sL-1} = p(T) W_0 with p(x) = x^(sL-1) mod phi(x) (phi: characteristic polynomial of the
// transition T; one tabulated polynomial per segment of a round, rt_mt_jump.h), evaluated without polynomial arithmetic as
//     W'[m] = XOR_{i : p_i = 1} y[i + m],   y = the raw words generated forward from W_0.
// T is singular: its kernel K is the low 31 bits of a window's first word (they never influence
// later words).  Writing W_0 = v + k (v in Im T, k in K), p(T) W_0 = T^J v + p_0 k, so a jumped
// window is exact except the low 31 bits of its first word -- which a segment never outputs (its
// outputs start at least one word later) and never dumps.
//
// Rounds: one launch covers up to SEGS segments (SEGS * L words); the next round starts
// from the exact window at the last segment's end.  The final numpy state is the window that
// contains the last consumed word, dumped by the segment that generates it.
#pragma once
#include <stdint.h>

#include <vector>

#include "rt_mt_jump.h"

namespace rtmt {

constexpr int N = 624;
constexpr int M = 397;
constexpr uint32_t MATRIX_A = 0x9908B0DFu, UPPER = 0x80000000u, LOWER = 0x7FFFFFFFu;
constexpr int64_t L = (int64_t)1 << RT_MT_SEG_LOG2;  // words per segment
constexpr int SEGS = 256;                             // segments per round (one jump polynomial each)
constexpr int POLY_BITS = 19937;

#if defined(__HIPCC__)
#define RT_MT_HD __host__ __device__ __forceinline__
#else
#define RT_MT_HD inline
#endif

RT_MT_HD uint32_t next_word(uint32_t xk, uint32_t xk1, uint32_t xkm) {
    const uint32_t y = (xk & UPPER) | (xk1 & LOWER);
    return xkm ^ (y >> 1) ^ ((y & 1u) ? MATRIX_A : 0u);
}

RT_MT_HD uint32_t temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9D2C5680u;
    y ^= (y << 15) & 0xEFC60000u;
    y ^= y >> 18;
    return y;
}

// numpy legacy random_sample: ((a >> 5) * 67108864 + (b >> 6)) / 9007199254740992
RT_MT_HD double to_double(uint32_t w0, uint32_t w1) {
    return ((double)(w0 >> 5) * 67108864.0 + (double)(w1 >> 6)) / 9007199254740992.0;
}

// jump polynomial of segment s in [1, SEGS) of a round: x^(sL-1), the window at s*L - 1 from the
// round's key window
inline const uint32_t* jump_poly(int s) { return RT_MT_JD[s - 1]; }

// the whole table as one array (device upload): (SEGS - 1) x 624 words
inline const uint32_t* tables_flat() { return &RT_MT_JD[0][0]; }
constexpr int64_t TABLE_WORDS = (int64_t)(SEGS - 1) * N;

// absolute (round-relative) word index where segment s's window starts
RT_MT_HD int64_t window_start(int s) { return s == 0 ? 0 : (int64_t)s * L - 1; }

// ---- launch plan (host) -----------------------------------------------------------------------
struct Round {
    int pos;              // outputs of the round start at word `pos` of its key window
    int64_t words;        // words consumed in this round (outputs and skipped draws)
    int64_t double_base;  // index of the round's first double in the output
    int nseg;             // segments launched
    int64_t dump_at;      // round-relative index of the final state window, or -1
    bool chain;           // the last segment writes the next round's key window (at SEGS*L - 1)
};

struct Plan {
    std::vector<Round> rounds;
    int final_pos = 0;  // numpy position within the dumped window (1..624)
};

// n_words = 2 * (doubles drawn); pos in [0, 624]
inline Plan make_plan(int pos, int64_t n_words) {
    Plan P;
    const int64_t per_round = (int64_t)SEGS * L;
    std::vector<int64_t> offset;  // absolute index (from the caller's key window) of each round's key
    int64_t done = 0, off = 0;
    int rpos = pos;
    for (;;) {
        Round r{};
        r.pos = rpos;
        r.words = n_words - done < per_round ? n_words - done : per_round;
        r.double_base = done / 2;
        const bool last = done + r.words >= n_words;
        r.nseg = r.words > 0 ? (int)((r.words + L - 1) / L) : 1;
        r.dump_at = -1;
        r.chain = !last;
        P.rounds.push_back(r);
        offset.push_back(off);
        if (last) break;
        done += r.words;
        off += per_round - 1;  // the next key window starts at SEGS*L - 1 ...
        rpos += 1;             // ... one word before the next output
    }
    // numpy keeps the 624-word block (aligned to its original key) holding the last consumed word,
    // with pos in (0, 624]
    const int64_t abs_end = pos + n_words;
    const int64_t k = (abs_end + N - 1) / N - 1;
    const int64_t dump_abs = k * N;
    P.final_pos = (int)(abs_end - dump_abs);
    size_t ri = P.rounds.size() - 1;
    while (ri > 0 && offset[ri] > dump_abs) --ri;
    Round& r = P.rounds[ri];
    r.dump_at = dump_abs - offset[ri];
    // launch the segment that generates it: window_start(q) < dump_at <= window_start(q + 1)
    int q = 0;
    while (q + 1 < SEGS && window_start(q + 1) < r.dump_at) ++q;
    if (q + 1 > r.nseg) r.nseg = q + 1;
    return P;
}

// segment q of a round that dumps the window at d (see make_plan)
// (the round's last segment also takes every later d: its outputs run to SEGS*L + pos)
RT_MT_HD bool dumps(int s, int64_t d) {
    if (d < 0) return false;
    const bool lo = (s == 0) ? d >= 0 : window_start(s) < d;
    return lo && (d <= window_start(s + 1) || s == SEGS - 1);
}

// ---- jump polynomials for arbitrary distances (host) ----------------------------------------
// x^J mod phi by left-to-right square-and-shift over GF(2): squaring spreads the bits, and phi is
// sparse (~135 terms), so a reduction XORs each high 64-bit chunk back at the few term offsets.
// A frame of a fixed shape consumes a fixed number of words, so the window at the end of frame k
// (the next frame's key) is one jump from frame k's key: the pipelined generator of frame k+1 need
// not wait for frame k's whole generation (rt_kernels.hip, k_mt_jump end block).
constexpr int PW = 312;  // 64-bit words of a reduced polynomial (19968 bits >= 19937)
struct Gf2 {
    uint64_t w[2 * PW];  // products before reduction
};

inline const std::vector<int>& phi_terms() {  // exponents e < 19937 of phi's terms
    // (a magic static: initialised once even when several host threads make polynomials)
    static const std::vector<int> t = [] {
        std::vector<int> v;
        for (int i = 0; i < POLY_BITS; ++i)
            if ((RT_MT_PHI[i >> 5] >> (i & 31)) & 1u) v.push_back(i);
        return v;
    }();
    return t;
}

inline void gf2_xor_at(uint64_t* a, uint64_t c, int64_t off) {  // a ^= c << off (bits)
    const int64_t wi = off >> 6;
    const int sh = (int)(off & 63);
    a[wi] ^= c << sh;
    if (sh) a[wi + 1] ^= c >> (64 - sh);
}

// reduce a (degree < 2 * 19968) modulo phi, in place; the result occupies words [0, PW)
inline void gf2_reduce(Gf2& a) {
    const std::vector<int>& terms = phi_terms();
    for (int i = 2 * PW - 1; i >= POLY_BITS / 64; --i) {
        for (;;) {
            int64_t base = (int64_t)64 * i - POLY_BITS;  // bit j of word i sits at x^(19937 + base + j)
            uint64_t c = a.w[i];
            if (base < 0) c &= ~0ull << (-base);  // (the boundary word: only bits >= 19937)
            if (!c) break;
            a.w[i] ^= c;
            if (base < 0) {
                c >>= -base;
                base = 0;
            }
            for (int e : terms) gf2_xor_at(a.w, c, base + e);  // x^19937 = sum of the other terms
        }
    }
}

inline uint64_t gf2_spread32(uint32_t v) {  // bit j -> bit 2j
    uint64_t x = v;
    x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
    x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
    x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x << 2)) & 0x3333333333333333ull;
    x = (x | (x << 1)) & 0x5555555555555555ull;
    return x;
}

// x^J mod phi as 624 32-bit words (bit i = word i/32, bit i%32), the layout of RT_MT_JD
inline std::vector<uint32_t> xpow_mod(uint64_t J) {
    Gf2 r{};
    r.w[0] = 1;
    for (int b = 63; b >= 0; --b) {
        if (!(J >> b) && b > 0) continue;  // (skip leading zeros; x^0 = 1)
        Gf2 q{};
        for (int k = 0; k < PW; ++k) {
            q.w[2 * k] = gf2_spread32((uint32_t)r.w[k]);
            q.w[2 * k + 1] = gf2_spread32((uint32_t)(r.w[k] >> 32));
        }
        gf2_reduce(q);
        if ((J >> b) & 1) {
            for (int k = PW; k > 0; --k) q.w[k] = (q.w[k] << 1) | (q.w[k - 1] >> 63);
            q.w[0] <<= 1;
            gf2_reduce(q);
        }
        r = q;
    }
    std::vector<uint32_t> out(N);
    for (int k = 0; k < N; ++k) out[k] = (uint32_t)(r.w[k >> 1] >> (32 * (k & 1)));
    return out;
}

// Where the next frame's key window lies for a frame of n_words words: the final window of a
// generation from position pos is at word 624 floor((pos + n_words - 1) / 624) of its key window,
// one of two values over pos in [1, 624].  end_jump is a window position 1249 .. 1873 words before
// it for every pos (J = 624 m - 1 from the table's convention), so the end block jumps to J with
// x^J and generates at most four blocks to reach the final window; 0 when the frame is too short.
inline uint64_t end_jump(int64_t n_words) {
    const int64_t base = (int64_t)N * ((n_words - 1) / N);
    return base >= 2 * (int64_t)N + 1 ? (uint64_t)(base - 2 * N - 1) : 0;
}

// ---- serial reference (host test driver) ------------------------------------------------------
// raw words generated forward from window `w` (624 words, w[0] = word at absolute index `start`)
struct SerialStream {
    std::vector<uint32_t> x;  // x[i] = word at absolute start + i
    explicit SerialStream(const uint32_t* w) : x(w, w + N) {}
    uint32_t at(int64_t i) {
        while ((int64_t)x.size() <= i) {
            const int64_t k = (int64_t)x.size() - N;
            x.push_back(next_word(x[k], x[k + 1], x[k + M]));
        }
        return x[i];
    }
};

inline void jump_serial(const uint32_t* w, const uint32_t* poly, uint32_t* out) {
    SerialStream y(w);
    y.at(POLY_BITS + N);
    for (int m = 0; m < N; ++m) out[m] = 0u;
    for (int i = 0; i < POLY_BITS; ++i) {
        if (!((poly[i >> 5] >> (i & 31)) & 1u)) continue;
        for (int m = 0; m < N; ++m) out[m] ^= y.x[i + m];
    }
}

// numpy-equal doubles: out[0..n_out) from (key, pos), then n_skip more draws; final state returned
inline void uniforms_serial(const uint32_t* key, int pos, int64_t n_out, int64_t n_skip, double* out,
                            uint32_t* key_out, int* pos_out) {
    const Plan P = make_plan(pos, 2 * (n_out + n_skip));
    std::vector<uint32_t> rkey(key, key + N), next(N);
    for (const Round& r : P.rounds) {
        for (int s = 0; s < r.nseg; ++s) {
            std::vector<uint32_t> w(N);
            if (s == 0) {
                w = rkey;
            } else {
                jump_serial(rkey.data(), jump_poly(s), w.data());
            }
            SerialStream g(w.data());
            const int64_t ws = window_start(s);
            const int64_t lo = (int64_t)s * L + r.pos, hi = (int64_t)(s + 1) * L + r.pos;
            const int64_t end = r.pos + r.words;
            for (int64_t a = lo; a < hi && a < end; a += 2) {
                const int64_t d = r.double_base + (a - r.pos) / 2;
                if (d < n_out) out[d] = to_double(temper(g.at(a - ws)), temper(g.at(a + 1 - ws)));
            }
            if (r.chain && s == SEGS - 1)
                for (int m = 0; m < N; ++m) next[m] = g.at(window_start(SEGS) + m - ws);
            if (dumps(s, r.dump_at))
                for (int m = 0; m < N; ++m) key_out[m] = g.at(r.dump_at + m - ws);
        }
        rkey = next;
    }
    *pos_out = P.final_pos;
}

}  // namespace rtmt
