// halda_prims.hpp -- constants, diagnostic stamps, LDS slices and the wave / 16-lane-segment reductions (DPP row
// rotations, row broadcasts, ballots) every kernel uses.
// Part of libhalda's single translation unit: included by halda.hip inside its anonymous namespace
// (after halda.h); not a standalone header.
#pragma once

constexpr int kRows = 4;            // capacity rows per device (link, RAM/Metal cap, <= 2 VRAM)
constexpr int kMaxRowNnz = 8;       // widest HALDA row (cycle rows: 6 device cols + z + C)
constexpr double kSlackEps = 1e-9;  // a capacity row counts as met within 1e-9 layers (oracle: same)
constexpr double kInf = __builtin_huge_val();
constexpr int kK1MaxM = 64;         // widest fleet the k = 1 fast path takes (lane = device)

// screen verdicts: settled / k = 1 fast path / general kernel for k > 1 / general kernel for k = 1
// (fleets wider than kK1MaxM and the fast path's hand-backs) / general kernel on global-memory tables
// (set by the LDS general launches for instances beyond their slice)
enum { CLS_DONE = 0, CLS_K1 = 1, CLS_GEN = 2, CLS_GEN1 = 3, CLS_BIG = 4 };

// Diagnostic build only (-DHALDA_STAMPS): per-instance s_memtime stamps at the
// phase boundaries of the solve kernel, read back with halda_debug_stamps().
#ifdef HALDA_STAMPS
constexpr int kStampInst = 65536, kStamps = 12;
__device__ unsigned long long g_halda_stamps[kStampInst * kStamps];
// the k = 2 tables G / H of the k-slot kernel's fleets (tools/kslot_tables.py): [fleet][device][e]
constexpr int kDumpFleets = 4096, kDumpDev = 16, kDumpE = 32;
__device__ double g_halda_dump[kDumpFleets * kDumpDev * kDumpE * 2];
// the k-slot kernel's split-scan part 1: per (workgroup, slot) wave, shader cycles summed over the
// threshold scan's iterations per step of an event (tools/scan_prof.py)
constexpr int kScanProf = 64;  // 4 segments x 16
__device__ unsigned long long g_halda_scanprof[kStampInst * kScanProf];
#define HALDA_STAMP(k)                                                                                  \
    do {                                                                                                \
        if (lane == 0 && I.inst < kStampInst) g_halda_stamps[I.inst * kStamps + (k)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
// fused sweep: per-fleet stamps (slot 0..6 shader clock, 7/8 constant-rate clock at start / end);
// with -DHALDA_STAMPS_DP per-instance stamps of the table path instead (HALDA_TSTAMP, slots 0, 6-8)
#ifdef HALDA_STAMPS_DP
#define HALDA_SSTAMP(slot, v) do {} while (0)
#define HALDA_TSTAMP(slot)                                                                              \
    do {                                                                                                \
        if (lane == 0 && inst < kStampInst) g_halda_stamps[inst * kStamps + (slot)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define HALDA_SSTAMP(slot, v)                                                                           \
    do {                                                                                                \
        if (lane == 0 && f < kStampInst) g_halda_stamps[int64_t(f) * kStamps + (slot)] = (v);           \
    } while (0)
#define HALDA_TSTAMP(slot) do {} while (0)
#endif
// k-slot kernel: per (workgroup, slot) wave, slots 0..4 shader clock (start, records done, solved,
// after the barrier, pick done), 5 the constant-rate clock at start (the helper wave stamps nothing)
#define HALDA_KSTAMPW(slot, v)                                                                          \
    do {                                                                                                \
        const int64_t e_ = int64_t(blockIdx.x) * SA.n_slot + q;                                         \
        if (q < SA.n_slot && (threadIdx.x & 63) == 0 && e_ < kStampInst)                                \
            g_halda_stamps[e_ * kStamps + (slot)] = (v);                                                \
    } while (0)
#else
#define HALDA_SSTAMP(slot, v) \
    do {                      \
    } while (0)
#define HALDA_TSTAMP(slot) do {} while (0)
#define HALDA_STAMP(k) \
    do {               \
    } while (0)
#endif
#ifndef HALDA_KSTAMPW
#define HALDA_KSTAMPW(slot, v) do {} while (0)
#endif
// -DHALDA_STAMPS_DECODE: stamps 1..5 mark the round trips inside decode_k1 instead
#ifdef HALDA_STAMPS_DECODE
#define HALDA_DSTAMP(k) HALDA_STAMP(k)
#define HALDA_PSTAMP(k) do {} while (0)
#else
#define HALDA_DSTAMP(k) do {} while (0)
#define HALDA_PSTAMP(k) HALDA_STAMP(k)
#endif
// -DHALDA_STAMPS_DP: stamps 1..5 mark the steps of the general kernel's k > 1 DP pass instead
#ifdef HALDA_STAMPS_DP
#define HALDA_KSTAMP(k) HALDA_STAMP(k)
#define HALDA_GSTAMP(k) do {} while (0)
#else
#define HALDA_KSTAMP(k) do {} while (0)
#define HALDA_GSTAMP(k) HALDA_STAMP(k)
#endif

// ---------------------------------------------------------------- LDS slice
// One solve wave = one 64-thread workgroup with its own LDS slice (bytes):
//   rows   per device kRows x int2 {pack(kind + 1, u + 1, v + 1), K}
//   cyc    per device {r1w, r2w, rhs1, rhs2} (cycle-row w coefficients and rhs)
//   cost   per device objective entries {cw, cn, cs0..cs3}
//   cnt    per device row counter | have1 << 8 | have2 << 16
//   st0/1  per device ints (DP backtracking states, ping-pong)
//   rng    per DP-tree slot: finite range [lo, hi] of the node's sequence
//   inc    per device next increment (greedy exchange)
//   G      [i][e] table, row stride RS (odd), leaves of the DP tree; k = 1 reduces in place
//   H      [i][e] least cycle time (k > 1 only)
//   work   DP tree levels when the leaves must survive (k > 1 threshold scan)
//   split  DP tree argmin (uint16 e of the left subtree), ~2 M (R + 1) bytes
struct Slice {
    int64_t rows, cyc, cost, cnt, st0, st1, rng, inc, G, H, work, split, total;
};

__host__ __device__ inline int64_t align16(int64_t x) { return (x + 15) & ~int64_t(15); }

// tab / tab_kc count M * RS doubles (RS = R + 1 rounded up to odd)
__host__ __device__ inline Slice make_slice(int mmax, int r1max, int tab, int tab_kc) {
    Slice s;
    int64_t o = 0;
    const int64_t tmax = tab > tab_kc ? tab : tab_kc;
    s.rows = o;  o = align16(o + int64_t(mmax) * kRows * 8);
    s.cyc = o;   o = align16(o + int64_t(mmax) * 4 * 8);
    s.cost = o;  o = align16(o + int64_t(mmax) * 6 * 8);
    s.cnt = o;   o = align16(o + int64_t(mmax) * 4);
    s.st0 = o;   o = align16(o + int64_t(mmax) * 4);
    s.st1 = o;   o = align16(o + int64_t(mmax) * 4);
    s.rng = o;   o = align16(o + int64_t(mmax) * 8);
    s.inc = o;   o = align16(o + int64_t(mmax) * 8);
    s.G = o;     o = align16(o + tmax * 8);
    s.H = o;     o = align16(o + int64_t(tab_kc) * 8);
    s.work = o;  o = align16(o + (tab_kc > 0 ? (int64_t(tab_kc) / 2 + 2 * int64_t(r1max) + 2) * 8 : 0));
    s.split = o; o = align16(o + (int64_t(mmax) + 12) * r1max * 2);
    s.total = o;
    return s;
}

__device__ inline void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// Wave reductions over the active lanes (DPP, result uniform) from the device library.
extern "C" __device__ double __ockl_wfred_min_f64(double);
extern "C" __device__ double __ockl_wfred_max_f64(double);
extern "C" __device__ int __ockl_wfred_min_i32(int);
extern "C" __device__ int __ockl_wfred_or_i32(int);
extern "C" __device__ int __ockl_wfred_add_i32(int);
// v_min_f64 / v_max_f64 as they are: for the non-signalling operands here they equal fmin / fmax
// (a quiet NaN operand yields the other), without the canonicalising v_max_f64 x, x, x the compiler
// puts in front of every fmin / fmax of a shuffled value.
__device__ inline double vmin_f64(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ inline double vmax_f64(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
template <int R>
__device__ inline double ror16(double v);
// min / max over the wave on every lane, without LDS or readlane: permlane swaps across the halves
// and rows, then DPP row rotations (min and max are exact: any order gives the same value)
// GFX9 DPP row broadcasts of a double (rows outside row_mask keep `old`): row_bcast:15 (0x142) gives
// rows 1 / 3 lane 15 / 47, row_bcast:31 (0x143) gives rows 2 / 3 lane 31.
template <int Ctrl, int RowMask>
__device__ inline double dpp_bcast_f64(double old, double v) {
    const uint64_t o = __builtin_bit_cast(uint64_t, old), u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = uint32_t(__builtin_amdgcn_update_dpp(int(uint32_t(o)), int(uint32_t(u)), Ctrl, RowMask, 0xf, false));
    const uint32_t hi = uint32_t(__builtin_amdgcn_update_dpp(int(uint32_t(o >> 32)), int(uint32_t(u >> 32)), Ctrl, RowMask, 0xf, false));
    return __builtin_bit_cast(double, (uint64_t(hi) << 32) | lo);
}
__device__ inline double bcast(double v, int src);
// min / max over the wave, uniform: every row reduced by DPP rotations, the rows combined by the
// row broadcasts (lane 63 ends up with all four), read from lane 63 (min and max are exact: any
// order gives the same value). Every lane must be active.
__device__ inline double wave_min(double v) {
    v = vmin_f64(v, ror16<8>(v));
    v = vmin_f64(v, ror16<4>(v));
    v = vmin_f64(v, ror16<2>(v));
    v = vmin_f64(v, ror16<1>(v));
    v = vmin_f64(v, dpp_bcast_f64<0x142, 0xa>(v, v));
    v = vmin_f64(v, dpp_bcast_f64<0x143, 0xc>(v, v));
    return bcast(v, 63);
}
__device__ inline double wave_max(double v) {
    v = vmax_f64(v, ror16<8>(v));
    v = vmax_f64(v, ror16<4>(v));
    v = vmax_f64(v, ror16<2>(v));
    v = vmax_f64(v, ror16<1>(v));
    v = vmax_f64(v, dpp_bcast_f64<0x142, 0xa>(v, v));
    v = vmax_f64(v, dpp_bcast_f64<0x143, 0xc>(v, v));
    return bcast(v, 63);
}
__device__ inline int wave_imin(int v) { return __ockl_wfred_min_i32(v); }
__device__ inline int wave_or(int v) { return __ockl_wfred_or_i32(v); }
__device__ inline int wave_sum(int v) { return __ockl_wfred_add_i32(v); }
// Record of lane `src` broadcast to the whole wave (src wave-uniform).
__device__ inline double bcast(double v, int src) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = __builtin_amdgcn_readlane(int(uint32_t(u)), src);
    const uint32_t hi = __builtin_amdgcn_readlane(int(uint32_t(u >> 32)), src);
    return __builtin_bit_cast(double, (uint64_t(hi) << 32) | lo);
}
__device__ inline int bcast(int v, int src) { return __builtin_amdgcn_readlane(v, src); }

// Sum over the wave in a fixed order, uniform: each 16-lane row all-reduced by DPP row rotations by
// 8, 4, 2, 1 (row16_reduce's steps: every lane of a row holds its row sum S_r), then
// (S3 + S2) + (S1 + S0) by the GFX9 row broadcasts, read from lane 63. With data in row 0 only (a
// problem of <= 16 devices) the result is S0 exactly, the bits of row16_reduce (Seg<16>). Every lane
// must be active.
__device__ inline double wave_sum_f64(double v) {
    v = v + ror16<8>(v);
    v = v + ror16<4>(v);
    v = v + ror16<2>(v);
    v = v + ror16<1>(v);
    v = v + dpp_bcast_f64<0x142, 0xa>(v, v);  // rows 1 / 3: S1 + S0, S3 + S2 (rows 0 / 2 unused)
    v = v + dpp_bcast_f64<0x143, 0xc>(v, v);  // row 3: (S3 + S2) + (S1 + S0)
    return bcast(v, 63);
}

// Row rotation of a 16-lane DPP row (row_ror:R, R = 1..15): lane i reads lane (i + R) mod 16 of its row.
template <int R>
__device__ inline int ror16(int v) {
    return __builtin_amdgcn_mov_dpp(v, 0x120 + R, 0xf, 0xf, true);
}
template <int R>
__device__ inline double ror16(double v) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = uint32_t(ror16<R>(int(uint32_t(u)))), hi = uint32_t(ror16<R>(int(uint32_t(u >> 32))));
    return __builtin_bit_cast(double, (uint64_t(hi) << 32) | lo);
}
// All-reduce over a 16-lane row by rotations 8, 4, 2, 1: after the first step a lane's value depends
// on its index mod 8 only, so lane i's partner (i + 4) mod 16 holds what its xor partner i ^ 4 holds,
// and so on: the same operands in the same order as the xor butterfly, and, op being commutative,
// the same bits on every lane of the row.
template <class T, class Op>
__device__ inline T row16_reduce(T v, Op op) {
    v = op(v, ror16<8>(v));
    v = op(v, ror16<4>(v));
    v = op(v, ror16<2>(v));
    v = op(v, ror16<1>(v));
    return v;
}

// Lanes per problem: Seg<64> = the whole wave (reductions, ballots and broadcasts as above);
// Seg<16> = four problems per wave, each on a 16-lane DPP row (row rotations for the reductions,
// ballots shifted to the row, broadcasts are bpermutes from the row). Sums over a 16-device problem
// are bit-identical either way: the 64-lane xor butterfly first adds the zeros of lanes 16..63
// (exact), then runs the steps 8, 4, 2, 1 that row16_reduce reproduces. Every lane of an active
// segment must be active.
template <int S_>
struct Seg {
    static_assert(S_ == 64 || S_ == 16, "a problem spans the wave or one 16-lane DPP row");
    static constexpr int S = S_;
    int sl, base;
    __device__ explicit Seg(int lane) : sl(S_ == 64 ? lane : (lane & (S_ - 1))), base(S_ == 64 ? 0 : (lane & ~(S_ - 1))) {}
    __device__ inline uint64_t bits(bool p) const {
        const uint64_t b = __ballot(p);
        if constexpr (S_ == 64) return b;
        else return (b >> base) & ((uint64_t(1) << S_) - 1);
    }
    __device__ inline int lowest(bool p) const {
        const uint64_t b = bits(p);
        return b ? __builtin_ctzll(b) : 0x7fffffff;
    }
    __device__ inline int highest(bool p) const {
        const uint64_t b = bits(p);
        return b ? 63 - __builtin_clzll(b) : -1;
    }
    __device__ inline double min_f64(double v) const {
        if constexpr (S_ == 64) return wave_min(v);
        else return row16_reduce(v, [](double a, double b) { return vmin_f64(a, b); });
    }
    __device__ inline double max_f64(double v) const {
        if constexpr (S_ == 64) return wave_max(v);
        else return row16_reduce(v, [](double a, double b) { return vmax_f64(a, b); });
    }
    __device__ inline double sum_f64(double v) const {
        if constexpr (S_ == 64) return wave_sum_f64(v);
        else return row16_reduce(v, [](double a, double b) { return a + b; });
    }
    __device__ inline int sum_i(int v) const {
        if constexpr (S_ == 64) return wave_sum(v);
        else return row16_reduce(v, [](int a, int b) { return a + b; });
    }
    __device__ inline bool any(bool p) const { return bits(p) != 0; }  // a ballot, no reduction
    __device__ inline int or_i(int v) const {
        if constexpr (S_ == 64) return wave_or(v);
        else return row16_reduce(v, [](int a, int b) { return a | b; });
    }
    __device__ inline int imin(int v) const {
        if constexpr (S_ == 64) return wave_imin(v);
        else return row16_reduce(v, [](int a, int b) { return min(a, b); });
    }
    __device__ inline double bcast(double v, int src) const {
        if constexpr (S_ == 64) return ::bcast(v, src);
        else return __shfl(v, base + src);
    }
    __device__ inline int bcast(int v, int src) const {
        if constexpr (S_ == 64) return ::bcast(v, src);
        else return __shfl(v, base + src);
    }
    // value of the previous lane of the segment (its first lane: its own): DPP wave_shr:1 / row_shr:1
    // with the lane's own value where there is no source lane
    __device__ inline double up1(double v) const {
        constexpr int ctrl = S_ == 64 ? 0x138 : 0x111;
        const uint64_t u = __builtin_bit_cast(uint64_t, v);
        const uint32_t lo = uint32_t(u), hi = uint32_t(u >> 32);
        const uint32_t l2 = uint32_t(__builtin_amdgcn_update_dpp(int(lo), int(lo), ctrl, 0xf, 0xf, false));
        const uint32_t h2 = uint32_t(__builtin_amdgcn_update_dpp(int(hi), int(hi), ctrl, 0xf, 0xf, false));
        return __builtin_bit_cast(double, (uint64_t(h2) << 32) | l2);
    }
};
using Wave = Seg<64>;
