// rt_mt_kernel.h -- the device generator of numpy's legacy `np.random.rand` stream (rt_mt.h):
// k_mt_y, k_mt_jump (segment start windows by jump polynomials) and k_mt_gen (the segments' words,
// tempered to doubles).  Included by rt_kernels.hip (the library) and tools/mt_jump_bench.cpp (a
// stand-alone timing harness).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <climits>

#include "rt_mt.h"

namespace rtmt_dev {

// wave priority of the generation kernels (s_setprio 0..3; the trace waves run at 0): a generator
// workgroup placed on a CU beside trace blocks issues ahead of them, finishes sooner and hands the
// CU's trace slot back sooner.  Same box, ex1 1080p pipelined frames: 0.938 -> 0.903 ms at 3
// (profiles/r05_mt_generator_ab.txt)
#ifndef MT_WAVE_PRIO
#define MT_WAVE_PRIO 3
#endif

struct MtArgs {
    const uint32_t* key;   // the round's key window (624 words)
    const uint32_t* tab;   // jump polynomials x^(sL-1), s = 1..SEGS-1 (624 words each)
    double* out;           // doubles of the whole call
    uint32_t* chain_dst;   // next round's key window (written by segment SEGS-1) or null
    uint32_t* dump_dst;    // final numpy key window or null
    int64_t words;         // words consumed by this round
    int64_t double_base;   // first double of this round
    int64_t n_out;         // doubles to write (the rest are skipped draws)
    int64_t dump_at;       // round-relative start of the final state window, or -1
    int64_t plane;         // doubles per jitter plane (0: write every double)
    int32_t plane_mask;    // bit k set: write the doubles of planes with index % 4 == k
    int32_t pos;           // outputs start at word `pos` of the key window
    const uint32_t* end_poly;  // x^end_at mod phi: k_mt_jump's last block makes the final window (dump_dst)
    int64_t end_at;            // window position of that jump
    int32_t key_in_win;        // the key window is copied to win[0] by k_mt_jump (segment 0 reads it there)
    int32_t compact;           // band mode: doubles stored at the segment's local offset (bands[4 s + 3])
    // y: the MT_YBLOCKS x 624 raw words generated from the key window (k_mt_y, or the previous
    // frame's end block), read by every jump block instead of each block generating them itself
    const uint32_t* y;
    uint32_t* y_next;     // end block: the y of the final window (the next frame's key), or null
    // band mode (a shard's rows): segment s covers bands[4 s + 1] doubles from double bands[4 s] of
    // the call (runs of rows of one jitter plane), jumped to by tab[s] = x^(2 bands[4 s] - 1) mod
    // phi (host-made per frame shape); its window is win[s + 1] (win[0]: the key).  bands[4 s + 2]
    // != 0: several runs merged, the segment generates through the other ranks' rows between them
    // and stores double k only where k % band_period < band_len.  With `compact` the doubles go to
    // the shard's own layout -- [sample][plane][its rows][width], from out + bands[4 s + 3], a merged
    // segment's band j of band_len doubles right after band j - 1 -- instead of the whole frame's
    // (a shard stores 1/N of the frame's jitter).  Null: the tabulated 2^19-word segments.
    const int64_t* bands;
    int64_t band_len, band_period;
    // jump parts: each window (a segment's, the end window) is made by `parts` blocks, each XOR-ing
    // 1/parts of the polynomial's terms into it with atomics (the segment windows are zeroed before
    // the launch); the end window accumulates in end_acc, and the end part that arrives last
    // (end_cnt) generates on from it
    uint32_t* end_acc;  // [624], zero between generations (the last end part leaves it so)
    uint32_t* end_cnt;  // zero between generations
    int32_t parts;      // MT_MIN_PARTS .. MT_MAX_PARTS; the launch's LDS is mt_jump_lds_bytes(parts)
    int32_t pad_;
};

// Launches per round (k_mt_y only when no earlier end block made the key's y).
//  k_mt_y: one workgroup: y = the 34 x 624 raw words generated from the key window, to HBM.
//  k_mt_jump: one workgroup per segment s >= 1 that has anything to store.  y (HBM -> LDS), then
//    W'[m] = XOR_{i : p_i} y[i + m] -- wave v of 8 takes coefficient words [78 v, 78 v + 78) (held
//    one per lane, read out by v_readlane), lane g the eleven outputs m = 11 g .. 11 g + 10 with y[32 w + 11 g .. + 42] in registers
//    (single-word LDS reads: the odd lane stride is free of bank conflicts); each coefficient bit is
//    one v_bitop3 acc ^= y & mask per output, branch-free; the waves' partial windows are XOR-reduced
//    through LDS and written to the window table.
//  k_mt_gen: MT_GEN_THREADS per segment.  A ring of three 624-word blocks in LDS; the next block is
//    made in three dependent stages of 227 / 227 / 170 words (x_{k+624} = x_{k+397} ^ twist(x_k,
//    x_{k+1}): stage two and three take their x_{k+397} from the thread's own earlier word) while the
//    current block's 312 doubles are tempered and stored.  7.5 KB of LDS and five waves per segment:
//    the trace kernels of the previous frame keep the rest of the CU.
// 8 waves.  A jump block alone takes 111 us (16 waves: 74 us), but it must find room next to the
// trace kernels of the frames in flight: a 16-wave block needs more registers per SIMD than one
// finished trace block frees and waited up to 2.5 ms for whole CUs to drain.  Same box, ex1 1080p
// pipelined frames, ms/frame (3 x 100 frames): 8 waves + high-priority generation stream 1.64,
// 16 waves 1.70, 8 waves 1.80, 16 waves + high-priority stream 1.85; one rank of 8 (3 x 400 frames,
// generation on the frame's stream): 8 waves 0.344, 16 waves 0.355 (tools/_gpu_cmd.sh A/B runs).
#ifdef MT_THREADS_OVERRIDE  // (experiments)
constexpr int MT_THREADS = MT_THREADS_OVERRIDE;
#else
constexpr int MT_THREADS = 512;
#endif
// blocks per jump (1/parts of the coefficient words each): a whole jump on one block took ~110 us
// of a CU; the frame-to-frame chain (each frame's key is the previous frame's end window) waited for
// the slowest block of the jump kernel.  A part loads only the slice of y its coefficient words
// read, so its LDS (and HBM read) shrinks with the part.
constexpr int MT_MAX_PARTS = 8;
constexpr int MT_MIN_PARTS = 2;
constexpr int MT_WAVES = MT_THREADS / 64;
constexpr int MT_G = 11;  // window outputs per lane in the jump (odd: conflict-free LDS reads; 57 lanes cover 624)
constexpr int MT_YBLOCKS = 34;                        // 21216 words >= 32 * 623 + 10 * 63 + 42
constexpr int MT_RED = 704;                           // per-wave stride of the reduction buffer (64 x 11)
static_assert(rtmt::N / MT_MIN_PARTS / MT_WAVES + 1 <= 64, "a wave's coefficient words fit one per lane");
static_assert(32 * (rtmt::N - 1) + MT_G * 63 + 32 + MT_G <= MT_YBLOCKS * rtmt::N, "jump window reads stay in y");
// y words a part of coefficient words [cw0, cw0 + n) reads: y[32 cw0 ..), 32 n + the lanes' reach,
// rounded up to whole uint4
__host__ __device__ constexpr int mt_yslice_words(int n) { return (32 * n + MT_G * 63 + 32 + MT_G + 3) & ~3; }
constexpr int MT_RED_WORDS = MT_WAVES * MT_RED + 3 * rtmt::N;  // the reduction, then the end ring
__host__ __device__ constexpr int mt_jump_lds_words(int parts) {
    return mt_yslice_words(rtmt::N / parts + 1) > MT_RED_WORDS ? mt_yslice_words(rtmt::N / parts + 1) : MT_RED_WORDS;
}
constexpr size_t MT_LDS_BYTES = (size_t)mt_jump_lds_words(MT_MIN_PARTS) * 4;  // the largest launch
inline size_t mt_jump_lds_bytes(int parts) { return (size_t)mt_jump_lds_words(parts) * 4; }
// generator threads per segment: 5 waves (227 make the next block, 312 store the current one).
// Measured (222 segments, ex1 1080p pinhole planes): 1 wave 1.17 ms, 4 waves 0.64, 5 waves 0.50,
// 8 waves 0.50 -- one wave is VALU-issue bound (~3000 cycles per 624-word block).  Round 5, with the
// one-range store test per block: one wave 281 us against 131 us per synchronous ex1 frame (2^17-word
// segments), and pipelined frames 1.60 against 0.99 ms (profiles/r05_mt_generator_ab.txt)
#ifdef MT_GEN_THREADS_OVERRIDE  // (experiments)
constexpr int MT_GEN_THREADS = MT_GEN_THREADS_OVERRIDE;
#else
constexpr int MT_GEN_THREADS = 320;
#endif

// workgroup barrier for LDS hand-offs only: waits for this wave's LDS traffic, not for its global
// stores (__syncthreads() would also drain the output stores)
__device__ __forceinline__ void mt_barrier() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0), vmcnt/expcnt untouched
    __builtin_amdgcn_s_barrier();
}

// block n (624 words) from block p by a workgroup.  Thread t < 227 makes words t, 227 + t and 454 + t:
// each needs only block p and the thread's own earlier word, so no barrier is needed inside the
// block; word 623 also needs word 0 of block n, which thread 169 recomputes.
__device__ __forceinline__ void mt_next_block(const uint32_t* p, uint32_t* n, int t) {
    if (t < 227) {
        const uint32_t a0 = p[t], a1 = p[t + 1], a2 = p[t + 397], b0 = p[227 + t], b1 = p[228 + t];
        const uint32_t c0 = t < 170 ? p[454 + t] : 0u;
        uint32_t c1 = t < 169 ? p[455 + t] : 0u;
        const uint32_t wa = rtmt::next_word(a0, a1, a2);
        const uint32_t wb = rtmt::next_word(b0, b1, wa);
        n[t] = wa;
        n[227 + t] = wb;
        if (t == 169) c1 = rtmt::next_word(p[0], p[1], p[397]);  // word 0 of block n
        if (t < 170) n[454 + t] = rtmt::next_word(c0, c1, wb);
    }
}

// What segment s of a round stores and generates (uniform over the segment's threads).
struct MtSeg {
    int64_t ws;       // round-relative index of the segment's window
    int64_t lo;       // first output word
    int64_t dbase;    // double of pair 0
    int64_t obase;    // where pair 0 is stored (out + obase; band mode compact: the local offset)
    int64_t gen_end;  // words to generate (exclusive)
    int64_t chain_at;
    int kend;         // pairs [0, kend) are stored (minus the planes outside plane_mask)
    bool chain, dump;
    bool masked;      // band mode, merged runs: only k % band_period < band_len is stored
    __device__ bool idle() const { return kend == 0 && !chain && !dump; }
};

__device__ __forceinline__ MtSeg mt_seg(const MtArgs& A, int s) {
    MtSeg g;
    g.masked = false;
    if (A.bands) {
        const int64_t d0 = A.bands[4 * s];
        g.ws = d0 == 0 ? 0 : 2 * d0 - 1;
        g.lo = 2 * d0 + A.pos;
        g.dbase = A.double_base + d0;
        g.obase = A.compact ? A.bands[4 * s + 3] : g.dbase;
        g.kend = (int)A.bands[4 * s + 1];
        g.masked = A.bands[4 * s + 2] != 0;
        g.gen_end = g.lo + 2 * (int64_t)g.kend;
        g.chain = g.dump = false;
        g.chain_at = 0;
        return g;
    }
    g.ws = rtmt::window_start(s);
    const int64_t end = A.pos + A.words;  // round-relative, exclusive
    g.lo = (int64_t)s * rtmt::L + A.pos;
    const int64_t hi = min((int64_t)(s + 1) * rtmt::L + A.pos, end);
    const int64_t npairs = hi > g.lo ? (hi - g.lo) / 2 : 0;
    g.dbase = A.double_base + (g.lo - A.pos) / 2;
    g.obase = g.dbase;
    // a skipped draw (beyond n_out, or in a plane outside plane_mask) is only stepped over
    const int kmax = (int)max<int64_t>(0, min<int64_t>(npairs, A.n_out - g.dbase));
    g.kend = kmax;
    if (A.plane > 0 && kmax > 0) {
        g.kend = 0;
        for (int64_t pi = g.dbase / A.plane; pi * A.plane < g.dbase + kmax; ++pi)
            if ((A.plane_mask >> (pi & 3)) & 1) g.kend = (int)min<int64_t>(kmax, (pi + 1) * A.plane - g.dbase);
    }
    g.gen_end = g.lo + 2 * (int64_t)g.kend;
    g.chain = A.chain_dst && s == rtmt::SEGS - 1;
    g.chain_at = rtmt::window_start(rtmt::SEGS);
    if (g.chain) g.gen_end = max(g.gen_end, g.chain_at + rtmt::N);
    g.dump = A.dump_dst && rtmt::dumps(s, A.dump_at);
    if (g.dump) g.gen_end = max(g.gen_end, A.dump_at + rtmt::N);
    return g;
}

// The raw words y = W_0, T W_0, ... (MT_YBLOCKS blocks of 624) from the key window, for the jump
// blocks of a generation: one workgroup, two LDS blocks ping-ponged.
__global__ __launch_bounds__(MT_THREADS) void k_mt_y(const uint32_t* key, uint32_t* y) {
    __shared__ uint32_t buf[2 * rtmt::N];
    const int t = threadIdx.x;
    for (int m = t; m < rtmt::N; m += MT_THREADS) buf[m] = y[m] = key[m];
    __syncthreads();
    for (int q = 0; q + 1 < MT_YBLOCKS; ++q) {
        const uint32_t* p = buf + (q & 1) * rtmt::N;
        uint32_t* n = buf + ((q + 1) & 1) * rtmt::N;
        mt_next_block(p, n, t);
        mt_barrier();
        for (int m = t; m < rtmt::N; m += MT_THREADS) y[(int64_t)(q + 1) * rtmt::N + m] = n[m];
    }
}

// Jump units, A.parts blocks each (block b: unit b / parts, part b % parts).  Tabulated mode:
// unit s - 1 makes the window of segment s >= 1 into win + 624 s.  Band mode (A.bands): unit s makes
// segment s's window into win + 624 (s + 1) (none for a band at the call's first double: it starts
// from the key).  The windows are XOR-accumulated by their parts with atomics into the zeroed table.
// With A.end_poly unit 0 (dispatched first: the next frame's generation waits for it, the segment
// windows only this frame's generators) jumps to the window at A.end_at (into A.end_acc), the
// segment units follow it, and its part that arrives last generates forward to the final window (A.dump_at), written to A.dump_dst -- the
// next frame's key, ready when this kernel ends (its whole generation need not have run) -- and on
// to the y of that window (A.y_next), so the next frame's jump blocks need no k_mt_y.  Block 0 also
// copies the key window to win[0] for the generators that start from it.
__global__ __launch_bounds__(MT_THREADS) void k_mt_jump(MtArgs A, uint32_t* win) {
    if (MT_WAVE_PRIO) __builtin_amdgcn_s_setprio(MT_WAVE_PRIO);
    extern __shared__ uint32_t mt_lds[];  // mt_jump_lds_words(A.parts)
    __shared__ int last_part;
    uint32_t* yl = mt_lds;                    // this part's slice of y
    uint32_t* red = mt_lds;                   // MT_WAVES x MT_RED (aliases y once it is read)
    uint32_t* ring = mt_lds + MT_WAVES * MT_RED;  // end unit: 3 blocks after the reduction
    const int parts = A.parts;
    const int part = (int)blockIdx.x % parts;
    const bool end_block = A.end_poly && (int)blockIdx.x < parts;
    const int unit = (int)blockIdx.x / parts - (A.end_poly ? 1 : 0);  // segment unit (end unit: -1)
    const bool band = A.bands != nullptr;
    const int s = band ? unit : unit + 1;
    const int t = threadIdx.x;
    if (blockIdx.x == 0)
        for (int m = t; m < rtmt::N; m += MT_THREADS) win[m] = A.key[m];
    if (!end_block && (band ? A.bands[4 * s] == 0 : mt_seg(A, s).idle())) return;
    const uint32_t* poly = end_block ? A.end_poly : A.tab + (int64_t)(band ? s : s - 1) * rtmt::N;
    // this part's coefficient words [p_lo, p_lo + p_n) read y[32 p_lo ..) only: that slice to LDS
    const int p_lo = part * rtmt::N / parts, p_n = (part + 1) * rtmt::N / parts - p_lo;
    {
        const uint4* ys = reinterpret_cast<const uint4*>(A.y + 32 * p_lo);
        uint4* yq = reinterpret_cast<uint4*>(yl);
        const int n4 = min(mt_yslice_words(p_n), MT_YBLOCKS * rtmt::N - 32 * p_lo) / 4;
#ifndef MT_DBG_NOLOAD  // (timing harness only)
        for (int m = t; m < n4; m += MT_THREADS) yq[m] = ys[m];
#endif
    }
    __syncthreads();
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6), g = t & 63;
    // this wave's coefficient words: its share of the part's
    const int cw_lo = p_lo + wv * p_n / MT_WAVES, cw_n = p_lo + (wv + 1) * p_n / MT_WAVES - cw_lo;
    uint32_t acc[MT_G];
#pragma unroll
    for (int k = 0; k < MT_G; ++k) acc[k] = 0u;
    // per coefficient word: the lane's 43 words y[32 cw_i + 11 g + i] from LDS, then every set bit j
    // adds y[32 cw_i + j + 11 g + k] to the lane's eleven outputs k.  The wave's coefficient words
    // are held one per lane and read out by v_readlane.
    const uint32_t my_cw = g < cw_n ? poly[cw_lo + g] : 0u;
    // the lane's window slides by 32 words from one coefficient word to the next: its last 11 words
    // are the next window's first (loaded once); a zero word still slides the window
    uint32_t r[32 + MT_G];
    {
        const uint32_t* yp = yl + 32 * (cw_lo - p_lo) + MT_G * g;
#pragma unroll
        for (int k = 0; k < MT_G; ++k) r[32 + k] = yp[k];
    }
    for (int ci = 0; ci < cw_n; ++ci) {
        const int cw_i = cw_lo + ci;
        const uint32_t cw = __builtin_amdgcn_readlane(my_cw, ci);
        // y[32 cw_i + 11 g + i]: single-word loads, the odd lane stride keeps them free of bank conflicts
        const uint32_t* yp = yl + 32 * (cw_i - p_lo) + MT_G * g;
#pragma unroll
        for (int k = 0; k < MT_G; ++k) r[k] = r[32 + k];
#pragma unroll
        for (int k = MT_G; k < 32 + MT_G; ++k) r[k] = yp[k];
        if (cw == 0u) continue;
        // bit pairs: pattern 01 / 10 adds one shifted row, 11 both rows (one three-input XOR per
        // output either way; a uniform branch per pair).  Measured per jump block (tools/
        // mt_jump_bench.cpp, 204 bands): pairs with a pre-XORed pair row 74 us; a v_bitop3 acc ^= y &
        // mask per bit, branch-free, 117 us; a uniform branch per bit 108 us; nibbles (xor3 of two pair
        // rows) 172 us
#pragma unroll
        for (int j = 0; j < 32; j += 2) {
            const uint32_t pat = (cw >> j) & 3u;  // wave-uniform
            if (pat == 1u) {
#pragma unroll
                for (int k = 0; k < MT_G; ++k) acc[k] ^= r[j + k];
            } else if (pat == 2u) {
#pragma unroll
                for (int k = 0; k < MT_G; ++k) acc[k] ^= r[j + 1 + k];
            } else if (pat == 3u) {
#pragma unroll
                for (int k = 0; k < MT_G; ++k) acc[k] = __builtin_amdgcn_bitop3_b32(acc[k], r[j + k], r[j + 1 + k], 0x96);
            }
        }
    }
    __syncthreads();  // every wave is done reading y
#pragma unroll
    for (int k = 0; k < MT_G; ++k) red[wv * MT_RED + MT_G * g + k] = acc[k];
    __syncthreads();
    uint32_t* wdst = end_block ? A.end_acc : win + (int64_t)(band ? s + 1 : s) * rtmt::N;
    for (int m = t; m < rtmt::N; m += MT_THREADS) {
        uint32_t w = 0u;
#pragma unroll
        for (int v = 0; v < MT_WAVES; ++v) w ^= red[v * MT_RED + m];
        if (w) atomicXor(wdst + m, w);
    }
    if (!end_block) return;
    // end unit: the part that arrives last generates from the window at end_at until the final
    // window (and its y) is written, and leaves the accumulator and the counter zero
    __threadfence();
    __syncthreads();
    if (t == 0) last_part = atomicAdd(A.end_cnt, 1u) == (uint32_t)(parts - 1);
    __syncthreads();
    if (!last_part) return;
    __threadfence();
    for (int m = t; m < rtmt::N; m += MT_THREADS) ring[m] = atomicExch(A.end_acc + m, 0u);
    if (t == 0) atomicExch(A.end_cnt, 0u);
    __syncthreads();
    const int64_t stop = A.dump_at + (A.y_next ? (int64_t)MT_YBLOCKS * rtmt::N : (int64_t)rtmt::N);
    int slot = 0;
    for (int64_t b0 = A.end_at; b0 < stop; b0 += rtmt::N) {
        const uint32_t* cur = ring + slot * rtmt::N;
        const int next = slot == 2 ? 0 : slot + 1;
        if (b0 + rtmt::N < stop) mt_next_block(cur, ring + next * rtmt::N, t);
        for (int m = t; m < rtmt::N; m += MT_THREADS) {
            const int64_t x = b0 + m - A.dump_at;
            if (x >= 0 && x < rtmt::N) A.dump_dst[x] = cur[m];
            if (A.y_next && x >= 0 && x < (int64_t)MT_YBLOCKS * rtmt::N) A.y_next[x] = cur[m];
        }
        slot = next;
        mt_barrier();
    }
}

// NT threads per segment: generate from its window (the key for segment 0) and store its doubles.
// NT = 64: one wave (no workgroup barrier, the next block in three staged chunks); NT >= 256: the
// workgroup form (threads < 227 make three words each).  The window, once read, is zeroed for the
// next generation's jump parts to XOR into (no memset launch on the generation's critical path:
// behind the trace kernels of the frames in flight a 150 KB fill waited 36-133 us for a CU).
template <int NT>
__global__ __launch_bounds__(NT) void k_mt_gen(MtArgs A, uint32_t* win) {
    __shared__ uint32_t ring[3 * rtmt::N];
    if (MT_WAVE_PRIO) __builtin_amdgcn_s_setprio(MT_WAVE_PRIO);  // (ahead of the trace waves)
    const int s = blockIdx.x;
    const int lane = threadIdx.x;
    const MtSeg g = mt_seg(A, s);
    uint32_t* w0p = A.bands ? (g.ws == 0 ? win : win + (int64_t)(s + 1) * rtmt::N)
                            : (s == 0 && !A.key_in_win) ? nullptr : win + (int64_t)s * rtmt::N;
    if (g.idle()) {
        if (w0p)
            for (int m = lane; m < rtmt::N; m += NT) w0p[m] = 0u;
        return;
    }
    const uint32_t* src = w0p ? w0p : A.key;
    for (int m = lane; m < rtmt::N; m += NT) {
        ring[m] = src[m];
        if (w0p) w0p[m] = 0u;  // (each thread zeroes the words it read)
    }
    __syncthreads();
    // block q holds words ws + 624 q .. + 623 and stores the pairs whose second word it holds
    const int off0 = (int)(g.lo - g.ws);  // 1 .. 625 (s > 0) or pos (s == 0)
    const int c0 = -((off0 + 1) >> 1);    // pair index of block 0's first pair
    double* outp = A.out + g.obase;
    const bool cm = g.masked && A.compact;  // merged bands stored back to back
    // plane of pair k: pidx while k < kb, then pidx + 1 (a block's 312 pairs span at most two planes)
    int64_t pidx = 0, kb = INT64_MAX;
    if (A.plane > 0) {
        pidx = g.dbase / A.plane;
        kb = (pidx + 1) * A.plane - g.dbase;
    }
    int kq = c0;  // pair of block q's first thread slot
    int slot = 0, prev = 2, next = 1;
    for (int64_t b0 = g.ws; b0 < g.gen_end; b0 += rtmt::N) {
        const uint32_t* p = ring + slot * rtmt::N;
        uint32_t* n = ring + next * rtmt::N;
        if (NT >= 256) {
            if (b0 + rtmt::N < g.gen_end) mt_next_block(p, n, lane);
        } else if (b0 + rtmt::N < g.gen_end) {
            // stage 1: words j < 227; stage 2: 227 + j; stage 3: 454 + j (j < 170), chunk c = lane + 64 c
            uint32_t wa[4], wb[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int j = lane + 64 * c;
                const int jj = j < 227 ? j : 226;
                wa[c] = rtmt::next_word(p[jj], p[jj + 1], p[jj + 397]);
                wb[c] = rtmt::next_word(p[227 + jj], p[228 + jj], wa[c]);
            }
            const uint32_t n0 = __shfl(wa[0], 0);  // word 0 of block n (for word 623)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int j = lane + 64 * c;
                if (j < 227) {
                    n[j] = wa[c];
                    n[227 + j] = wb[c];
                }
                if (j < 170) n[454 + j] = rtmt::next_word(p[454 + j], j == 169 ? n0 : p[min(455 + j, 623)], wb[c]);
            }
        }
        if (kq >= kb) {
            ++pidx;
            kb += A.plane;
        }
        const uint32_t* cur = p;
        // the block's pairs k in [klo, khi) are all stored when no merged-band mask applies and the
        // (at most two) planes they lie in are stored planes: one range test per pair (the usual
        // block); otherwise every pair's plane and band are tested
        const int klo = max(kq, 0), khi = min(kq + 312, g.kend);
        bool every = !g.masked;
        if (every && A.plane > 0)
            every = (klo >= kb || ((A.plane_mask >> (int)(pidx & 3)) & 1)) &&
                    (khi <= kb || ((A.plane_mask >> (int)((pidx + 1) & 3)) & 1));
        if (every) {
#pragma unroll
            for (int i = 0; i < (312 + NT - 1) / NT; ++i) {
                const int t = lane + NT * i;
                const int k = kq + t;
                if (t < 312 && k >= klo && k < khi) {
                    const int o = off0 + 2 * (c0 + t);  // in-block offset of the pair's first word: -1 .. 622
                    const uint32_t x0 = o >= 0 ? cur[o] : ring[prev * rtmt::N + rtmt::N - 1];
                    const uint32_t x1 = cur[o + 1];
                    outp[k] = rtmt::to_double(rtmt::temper(x0), rtmt::temper(x1));
                }
            }
        } else {
#pragma unroll
            for (int i = 0; i < (312 + NT - 1) / NT; ++i) {
                const int t = lane + NT * i;
                const int k = kq + t;
                if (t < 312 && k >= 0 && k < g.kend &&
                    (A.plane == 0 || ((A.plane_mask >> (int)((k < kb ? pidx : pidx + 1) & 3)) & 1)) &&
                    (!g.masked || (uint32_t)k % (uint32_t)A.band_period < (uint32_t)A.band_len)) {
                    const int o = off0 + 2 * (c0 + t);
                    const uint32_t x0 = o >= 0 ? cur[o] : ring[prev * rtmt::N + rtmt::N - 1];
                    const uint32_t x1 = cur[o + 1];
                    const int64_t ko = cm ? (int64_t)((uint32_t)k / (uint32_t)A.band_period) * A.band_len +
                                                (uint32_t)k % (uint32_t)A.band_period
                                          : (int64_t)k;
                    outp[ko] = rtmt::to_double(rtmt::temper(x0), rtmt::temper(x1));
                }
            }
        }
        if (g.chain || g.dump) {
            for (int m = lane; m < rtmt::N; m += NT) {
                const int64_t x = b0 + m;
                const uint32_t v = cur[m];
                if (g.chain && x >= g.chain_at && x < g.chain_at + rtmt::N) A.chain_dst[x - g.chain_at] = v;
                if (g.dump && x >= A.dump_at && x < A.dump_at + rtmt::N) A.dump_dst[x - A.dump_at] = v;
            }
        }
        kq += 312;
        prev = slot;
        slot = next;
        next = next == 2 ? 0 : next + 1;
        // (one wave: its LDS operations complete in order, the barrier is nearly free; the output
        // stores are not waited for)
        mt_barrier();
    }
}

}  // namespace rtmt_dev
