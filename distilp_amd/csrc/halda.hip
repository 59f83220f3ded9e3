// libhalda — exact batched solver for fixed-k HALDA MILPs on MI355X (gfx950).
//
// Replaces the per-(fleet, k) call scipy.optimize.milp -> HiGHS made by the
// reference at src/distilp/solver/halda_p_solver.py:340-346; the C ABI is in
// include/halda.h, the design (and why the DP is exact) in DESIGN.md.
//
// A batch is solved by two launches on one stream:
//   screen   one wave per instance: validates the equality row and the
//            column bounds, settles bound-infeasible instances (sum lb(w) > W,
//            every k with M > L/k) and non-HALDA inputs right there, and
//            flags the rest (class 1: k = 1, class 2: k > 1);
//   solve    persistent 64-thread workgroups (= one wave each, no barriers),
//            each owning instances blockIdx + j * gridDim (a ballot over the
//            screen verdicts skips the settled ones), with its own LDS slice:
//            rows    decode the CSR rows (lane-strided) into per-device
//                    records in LDS, validating the HALDA pattern;
//            tables  lane = device: for every extra-layer count e in [0, R]
//                    (w = lb(w) + e, R = W - sum lb(w)) the best GPU split n
//                    (cost convex piecewise-linear in n -> only interval ends
//                    and slack kinks are evaluated): G[e][i] cost, H[e][i]
//                    least cycle time (k > 1 only);
//            DP      min-plus DP over sum(e) as a balanced tree of pairwise
//                    convolutions (lanes = (node, state) tasks), argmin splits
//                    kept for a parallel top-down backtrack; k > 1 adds a
//                    pruned ascending scan over cycle-time thresholds T;
//            output  lane = device rebuilds x for its chosen w.
// Floating point keeps the reference's operation order (-ffp-contract=off).

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "halda.h"

namespace {

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
constexpr int kStampInst = 65536, kStamps = 10;
__device__ unsigned long long g_halda_stamps[kStampInst * kStamps];
#define HALDA_STAMP(k)                                                                                  \
    do {                                                                                                \
        if (lane == 0 && I.inst < kStampInst) g_halda_stamps[I.inst * kStamps + (k)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
// slots 7..9 of the fused kernel's waves: shader clock at wave start, constant-rate
// (100 MHz) clock at wave start and at wave end
#define HALDA_WSTAMP(slot, v)                                                                           \
    do {                                                                                                \
        if (lane == 0 && inst < kStampInst) g_halda_stamps[inst * kStamps + (slot)] = (v);              \
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
// after the barrier, pick done), 5 the constant-rate clock at start
#define HALDA_KSTAMPW(slot, v)                                                                          \
    do {                                                                                                \
        const int64_t e_ = int64_t(blockIdx.x) * SA.n_slot + q;                                         \
        if ((threadIdx.x & 63) == 0 && e_ < kStampInst) g_halda_stamps[e_ * kStamps + (slot)] = (v);    \
    } while (0)
#elif defined(HALDA_MARKS)  // asm listing only: phase markers for tools/asm_regions.py
#define HALDA_SSTAMP(slot, v) asm volatile("; PHASE_MARK " #slot)
#define HALDA_TSTAMP(slot) do {} while (0)
#define HALDA_WSTAMP(slot, v) do {} while (0)
#define HALDA_STAMP(k) do {} while (0)
#else
#define HALDA_SSTAMP(slot, v) \
    do {                      \
    } while (0)
#define HALDA_TSTAMP(slot) do {} while (0)
#define HALDA_WSTAMP(slot, v) \
    do {                      \
    } while (0)
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


__device__ inline void write_done(const halda_result &R, int inst, int status, int64_t nodes) {
    R.status[inst] = status;
    R.nodes[inst] = nodes;
    R.obj_lin[inst] = kInf;
    R.dual_bound[inst] = status == HALDA_STATUS_INFEASIBLE ? kInf : -kInf;
    R.gap[inst] = kInf;
}

__host__ __device__ inline int odd_stride(int r1) { return r1 | 1; }

// ---------------------------------------------------------------- screen
// One wave screens kScreenPer consecutive instances. Settles everything
// decidable from the equality row and the w lower bounds (non-HALDA shape, bound
// infeasibility such as M > W = L/k) and flags the rest for the solve kernel
// (class 1: c[C] == 0, class 2: c[C] > 0). The loads of all its instances are
// issued together: headers (lane g = instance g), then equality-row extents and
// bounds (lane g), then per instance the equality row and w bounds (lane =
// device), so a wave spends three memory round trips on kScreenPer instances.
#ifndef HALDA_SCREEN_PER
#define HALDA_SCREEN_PER 8
#endif
constexpr int kScreenPer = HALDA_SCREEN_PER;

__device__ inline int64_t shfl64(int64_t v, int src) {
    const int lo = __shfl(int(uint32_t(uint64_t(v))), src), hi = __shfl(int(uint32_t(uint64_t(v) >> 32)), src);
    return int64_t((uint64_t(uint32_t(hi)) << 32) | uint32_t(lo));
}

// Per-lane outcome of screen_group: lane g < kScreenPer describes instance i0 + g.
struct ScreenOut {
    int N, m, verdict;
    int64_t co, ro, cs;
};

__device__ inline void screen_group(const halda_batch &B, const halda_result &Rz, uint8_t *cls, int64_t i0, int lane,
                                    int mmax, int r1max, int tab, int tab_kc, ScreenOut &so) {
    // lane g < kScreenPer: header of instance i0 + g. Loads are branch-free (lanes
    // without an instance read a valid element and discard it) so that each round
    // trip's loads issue before the first wait.
    const int64_t my = i0 + lane;
    const bool own = lane < kScreenPer && my < B.n_inst;
    const int64_t mc = own ? my : i0;
    const int N0 = B.n_cols[mc], m0 = B.n_rows[mc];
    const int64_t co0 = B.col_off[mc], ro0 = B.row_off[mc], cs0 = B.csr_off[mc];
    const int N = own ? N0 : 1, m = own ? m0 : 1;
    const int64_t co = own ? co0 : 0, ro = own ? ro0 : 0, cs = own ? cs0 : 0;
    int status = 0;  // 0 = still open
    if (N < 1 || (N - 1) % 7 != 0 || m < 1) status = HALDA_STATUS_UNSUPPORTED;
    const int M = status ? 0 : (N - 1) / 7;
    if (!status && M > mmax) status = HALDA_STATUS_TOO_LARGE;
    // round trip 2: equality-row extent and bounds, c[C] (lane g), and the w bounds of
    // every instance of the group (lane = device)
    const int ma = max(m0, 1);
    const int32_t *rp = B.row_ptr + cs0;
    const int eqs0 = rp[ma - 1], eqe0 = rp[ma];
    const double Wd0 = B.row_ub[ro0 + ma - 1], Wl0 = B.row_lb[ro0 + ma - 1];
    const double cC0 = B.c[co0 + 7 * int64_t(max(M, 0))];
    double lbv[kScreenPer];
    int Mg_[kScreenPer];
#pragma unroll
    for (int g = 0; g < kScreenPer; ++g) {
        const int Mg = __shfl(M, g);
        const int64_t cg = shfl64(co0, g);
        const int64_t idx = cg + (lane < Mg ? lane : 0);
        lbv[g] = B.col_lb[idx];  // w upper bounds are left to the solve
        Mg_[g] = Mg;
    }
    const bool live = own && !status;
    const int eqs = live ? eqs0 : 0, eqe = live ? eqe0 : 0;
    const double Wd = live ? Wd0 : 0.0, Wl = live ? Wl0 : 0.0, cC = live ? cC0 : 0.0;
    if (!status && (!(Wl == Wd) || !(Wd >= 0.0 && Wd < 1e6 && Wd == floor(Wd)) || eqe - eqs != M))
        status = HALDA_STATUS_UNSUPPORTED;

    // round trip 3: equality row entries per instance g (lane = device); lanes
    // without an entry read the first entry of an open instance's row (valid)
    int cv[kScreenPer];
    double vv[kScreenPer];
    const uint64_t open = __ballot(lane < kScreenPer && own && !status && M > 0);
    const int safe = open ? __shfl(eqs0, __builtin_ctzll(open)) : 0;
#pragma unroll
    for (int g = 0; g < kScreenPer; ++g) {
        const int stg = __shfl(status, g), eg = __shfl(eqs0, g);
        const bool in = open && i0 + g < B.n_inst && stg == 0 && lane < Mg_[g];
        const int idx = in ? eg + lane : safe;
        const int c0 = open ? B.col_idx[idx] : 0;
        const double v0 = open ? B.val[idx] : 1.0;
        cv[g] = in ? c0 : lane;
        vv[g] = in ? v0 : 1.0;
        if (!in) lbv[g] = 0.0;
    }
    int verdict = CLS_DONE, vstatus = status;  // lane g: outcome of instance g
#pragma unroll
    for (int g = 0; g < kScreenPer; ++g) {
        if (i0 + g >= B.n_inst) break;
        const int stg = __shfl(status, g);
        if (stg) continue;
        const int Mg = __shfl(M, g), eg = __shfl(eqs, g);
        const int64_t cg = shfl64(co, g);
        const double Wg = __shfl(Wd, g);
        int bad = 0, infeas = 0, sumlo = 0;
        auto one = [&](int i, int col, double v, double lb) {
            bad |= col != i || v != 1.0;
            const int wlo = int(ceil(lb));
            infeas |= wlo > int(Wg) || lb < 0.0;
            sumlo += wlo;
        };
        if (lane < Mg) one(lane, cv[g], vv[g], lbv[g]);
        for (int i = lane + 64; i < Mg; i += 64) one(i, B.col_idx[eg + i], B.val[eg + i], B.col_lb[cg + i]);
        bad = wave_or(bad | (infeas << 1));
        sumlo = wave_sum(sumlo);
        const int W = int(Wg);
        int st = 0, v = CLS_DONE;
        if (bad & 1) st = HALDA_STATUS_UNSUPPORTED;
        else if ((bad & 2) || sumlo > W || (Mg == 0 && W > 0)) st = HALDA_STATUS_INFEASIBLE;
        else if (Mg == 0) st = HALDA_STATUS_OPTIMAL;  // no devices and W = 0: x = [C = 0]
        else {
            const int R1 = W - sumlo + 1;
            const bool kc = __shfl(cC, g) > 0.0;
            if (R1 > r1max || int64_t(Mg) * odd_stride(R1) > (kc ? tab_kc : tab)) st = HALDA_STATUS_TOO_LARGE;
            else v = kc ? CLS_GEN : (Mg > kK1MaxM ? CLS_GEN1 : CLS_K1);
        }
        if (lane == g) {
            vstatus = st;
            verdict = v;
        }
    }
    so.N = N;
    so.m = m;
    so.co = co;
    so.ro = ro;
    so.cs = cs;
    so.verdict = own ? verdict : CLS_DONE;
    if (own) {
        cls[my] = uint8_t(verdict);
        if (verdict == CLS_DONE) {
            if (vstatus == HALDA_STATUS_OPTIMAL) {
                Rz.x[co] = 0.0;
                Rz.status[my] = HALDA_STATUS_OPTIMAL;
                Rz.obj_lin[my] = Rz.dual_bound[my] = Rz.gap[my] = 0.0;
                Rz.nodes[my] = 0;
            } else {
                write_done(Rz, int(my), vstatus, 0);
            }
        }
    }
}

// ---------------------------------------------------------------- solve
// One device's data in registers (lane = device). Rows are regrouped per
// slack: all rows of slack j share (u, v) (validated at decode; this is what
// keeps the cost L-natural convex), so they merge into one requirement
// s_j >= u_j w + v_j n + K_j with K_j the largest; pure (w, n) rows (the link
// n <= w) are the two "f" rows: u w + v n <= K.
struct Dev {
    double cw, cn, cs0, cs1, cs2, cs3, r1w, r2w, rhs1, rhs2;
    int wlo, whi, nlo, nhi;
    int slo[4], shi[4];
    int us[4], vs[4], Ks[4];
    int uf[2], vf[2], Kf[2];
};

constexpr int kNoRow = -(1 << 29);  // K of an absent row: never binds

// Least slacks for integer (w, n); false when a row or a slack bound cannot be met.
__device__ inline bool least_slacks(const Dev &d, int w, int n, int s[4]) {
    bool ok = d.uf[0] * w + d.vf[0] * n <= d.Kf[0] && d.uf[1] * w + d.vf[1] * n <= d.Kf[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        s[j] = max(d.slo[j], d.us[j] * w + d.vs[j] * n + d.Ks[j]);
        ok = ok && s[j] <= d.shi[j];
    }
    return ok;
}

// Objective contribution (same term order as c.x in the reference).
__device__ inline double dev_cost(const Dev &d, int w, int n, const int s[4]) {
    double g = d.cw * double(w);
    g = g + d.cn * double(n);
    g = g + d.cs0 * double(s[0]);
    g = g + d.cs1 * double(s[1]);
    g = g + d.cs2 * double(s[2]);
    g = g + d.cs3 * double(s[3]);
    return g;
}

// Cycle rows: C >= P + z, C >= Q - z, z >= 0  ->  least C = max(P, (P + Q) / 2).
__device__ inline void dev_cycle(const Dev &d, int w, int n, const int s[4], double &P, double &Q) {
    const double t0 = d.cn * double(n), t1 = d.cs0 * double(s[0]), t2 = d.cs1 * double(s[1]),
                 t3 = d.cs2 * double(s[2]), t4 = d.cs3 * double(s[3]);
    double a1 = d.r1w * double(w), a2 = d.r2w * double(w);
    a1 = a1 + t0; a1 = a1 + t1; a1 = a1 + t2; a1 = a1 + t3; a1 = a1 + t4;
    a2 = a2 + t0; a2 = a2 + t1; a2 = a2 + t2; a2 = a2 + t3; a2 = a2 + t4;
    P = a1 - d.rhs1;
    Q = a2 - d.rhs2;
}

__device__ inline double least_cycle(const Dev &d, int w, int n, const int s[4]) {
    double P, Q;
    dev_cycle(d, w, n, s, P, Q);
    return Q >= P ? 0.5 * (P + Q) : P;
}

// Feasible interval of n for w layers (from nlo/nhi, the pure rows and the slack upper bounds).
__device__ inline void n_interval(const Dev &d, int w, int &nL, int &nU) {
    nL = d.nlo;
    nU = d.nhi;
#pragma unroll
    for (int f = 0; f < 2; ++f) {
        const int rest = d.Kf[f] - d.uf[f] * w;  // v n <= rest
        if (d.vf[f] > 0) nU = min(nU, rest);
        if (d.vf[f] < 0) nL = max(nL, -rest);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int r = d.shi[j] - d.us[j] * w - d.Ks[j];  // v n <= r
        if (d.vs[j] > 0) nU = min(nU, r);
        if (d.vs[j] < 0) nL = max(nL, -r);
    }
}

__device__ inline void try_split(const Dev &d, int w, int nn, int nL, int nU, double &best, int &bn, int bs[4]) {
    nn = min(max(nn, nL), nU);
    int s[4];
    const bool ok = least_slacks(d, w, nn, s);
    const double g = dev_cost(d, w, nn, s);
    // branch-free: selects and non-short-circuit tests (the same update as "if ok and better")
    const bool better = ok & ((g < best) | ((g == best) & (nn < bn)));
    best = better ? g : best;
    bn = better ? nn : bn;
#pragma unroll
    for (int j = 0; j < 4; ++j) bs[j] = better ? s[j] : bs[j];
}

// Best GPU split n for w layers by full candidate search. The cost is convex
// piecewise-linear in integer n (each slack is max(lb, affine in n with slope
// -1/0/+1), prices >= 0), so its minimum over the feasible interval is at an
// end or at a kink. Ties -> smallest n.
__device__ inline bool split_full(const Dev &d, int w, double &g, int &n, int s[4]) {
    int nL, nU;
    n_interval(d, w, nL, nU);
    if (nL > nU) return false;
    double best = kInf;
    int bn = -1;
    try_split(d, w, nL, nL, nU, best, bn, s);
    try_split(d, w, nU, nL, nU, best, bn, s);
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (d.vs[j] != 0) try_split(d, w, d.vs[j] * (d.slo[j] - d.us[j] * w - d.Ks[j]), nL, nU, best, bn, s);
    if (bn < 0) return false;
    g = best;
    n = bn;
    return true;
}

__device__ inline bool split_first(const Dev &d, int w, double &g, int &n, int s[4]) { return split_full(d, w, g, n, s); }

// Incremental step w-1 -> w. The cost is L-natural convex in (w, n) (every term
// depends on w, n or w - n only; validated at decode), so the least minimiser
// moves by 0 or +1: only n_prev and n_prev + 1 are candidates.
__device__ inline bool split_step(const Dev &d, int w, int n_prev, double &g, int &n, int s[4]) {
    int nL, nU;
    n_interval(d, w, nL, nU);
    if (nL > nU) return false;
    double best = kInf;
    int bn = -1;
    try_split(d, w, n_prev, nL, nU, best, bn, s);
    try_split(d, w, n_prev + 1, nL, nU, best, bn, s);
    if (bn < 0) return false;
    g = best;
    n = bn;
    return true;
}

// Record accessors shared by the solve code (Dev here; the k-sweep's FieldRec has its own
// overloads, found by argument-dependent lookup where the templates are instantiated).
__device__ inline int rec_wlo(const Dev &d) { return d.wlo; }
__device__ inline int rec_whi(const Dev &d) { return d.whi; }

struct WaveCtx {
    int2 *rows;    // [i][q] packed capacity rows
    double *cyc;   // [i] {r1w, r2w, rhs1, rhs2}
    double *cost;  // [i] {cw, cn, cs0, cs1, cs2, cs3}
    int *cnt;
    int *st0, *st1;
    int2 *rng;     // [slot] finite range of a DP-tree node (merge path)
    double *inc;   // [i] next increment of device i (greedy exchange)
    double *G, *H, *work;
    uint16_t *split;
    uint8_t *dparg;  // register sweep: the wave's arg-min strip of the k = 1 DP fallback (k1_dp)
};

// Device record: costs / decoded rows from LDS, integer bounds from the batch.
__device__ inline void load_dev(Dev &d, const halda_batch &B, const WaveCtx &w, int64_t co, int M, int i,
                                double Wd) {
    const double *c = w.cost + 6 * i;
    d.cw = c[0]; d.cn = c[1]; d.cs0 = c[2]; d.cs1 = c[3]; d.cs2 = c[4]; d.cs3 = c[5];
    d.wlo = int(ceil(B.col_lb[co + i]));
    d.whi = int(floor(fmin(B.col_ub[co + i], Wd)));
    d.nlo = int(ceil(B.col_lb[co + M + i]));
    d.nhi = int(floor(fmin(B.col_ub[co + M + i], Wd)));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        d.slo[j] = int(ceil(B.col_lb[co + (2 + j) * M + i]));
        d.shi[j] = int(floor(fmin(B.col_ub[co + (2 + j) * M + i], 1e6)));
        d.us[j] = d.vs[j] = 0;
        d.Ks[j] = kNoRow;
    }
    d.uf[0] = d.vf[0] = d.uf[1] = d.vf[1] = 0;
    d.Kf[0] = d.Kf[1] = 0;
    const double *y = w.cyc + 4 * i;
    d.r1w = y[0]; d.r2w = y[1]; d.rhs1 = y[2]; d.rhs2 = y[3];
    const int nrow = w.cnt[i] & 0xff;
    int nf = 0;
#pragma unroll
    for (int q = 0; q < kRows; ++q) {
        if (q < nrow) {
            const int2 r = w.rows[i * kRows + q];
            const int kind = (r.x & 0xff) - 1, u = ((r.x >> 8) & 0xff) - 1, v = ((r.x >> 16) & 0xff) - 1;
            if (kind < 0) {
                if (nf == 0) { d.uf[0] = u; d.vf[0] = v; d.Kf[0] = r.y; }
                else { d.uf[1] = u; d.vf[1] = v; d.Kf[1] = r.y; }
                ++nf;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (kind == j) {
                    d.us[j] = u;
                    d.vs[j] = v;
                    d.Ks[j] = max(d.Ks[j], r.y);
                }
            }
        }
    }
}

struct LeafInfo {
    bool convex;  // every leaf's finite set is an interval and the leaf is convex on it
    bool empty;   // some leaf has no allowed entry (the call is infeasible)
    bool mono;    // every leaf's H is nondecreasing on its finite set
    int lo_sum;   // sum of the leaves' first allowed e
    int cap;      // sum of (hi - lo)
    int my_lo, my_hi;  // this lane's leaf range (device i = lane; M <= 64)
};

// Leaf pre-pass of one DP call (lane = device): finite range [lo, hi] of the
// leaf A_i[e] = G[i][e] (+inf where H[i][e] > T when use_T) into rng[i]. The
// cost is L-natural convex in (w, n), so G_i (its minimum over n) is convex in w
// and its threshold sublevel sets are intervals; the check guards the floating
// point (increments must not decrease by more than 1e-12 relative).
__device__ LeafInfo leaf_ranges(const WaveCtx &w, int M, int R1, int RS, bool use_T, double T, int lane,
                                bool want_mono = false) {
    bool ok = true, empty = false, mono = true;
    int lo_sum = 0, cap = 0, my_lo = R1, my_hi = -1;
    for (int i = lane; i < M; i += 64) {
        const double *G = w.G + int64_t(i) * RS, *H = w.H + int64_t(i) * RS;
        int lo = R1, hi = -1, cnt = 0;
        double prev = kInf, dprev = -kInf, hprev = -kInf;
        for (int e = 0; e < R1; ++e) {
            const double g = G[e];
            const double h = want_mono || use_T ? H[e] : 0.0;
            const bool in = g < kInf && (!use_T || h <= T);
            if (in) {
                if (cnt > 0) {
                    const double d = g - prev;
                    ok = ok && (hi == e - 1) && d >= dprev - 1e-12 * fmax(1.0, fabs(g));
                    dprev = d;
                }
                mono = mono && h >= hprev;
                hprev = h;
                lo = min(lo, e);
                hi = e;
                prev = g;
                ++cnt;
            }
        }
        empty = empty || cnt == 0;
        lo_sum += lo;
        cap += hi - lo;
        w.rng[i] = make_int2(lo, hi);
        if (i == lane) {
            my_lo = lo;
            my_hi = hi;
        }
    }
    LeafInfo li;
    li.mono = want_mono && !wave_or(!mono);
    li.my_lo = my_lo;
    li.my_hi = my_hi;
    li.convex = !wave_or(!ok);
    li.empty = wave_or(empty);
    li.lo_sum = wave_sum(lo_sum);
    li.cap = wave_sum(cap);
    return li;
}

// Run of the greedy round's winner over its table row G: increment 0 (its
// smallest, e0 -> e0 + 1) is taken, and increment t (e0 + t -> e0 + t + 1)
// follows while each of 1..t still beats the runner-up's m2 (ties go to the lower
// device index: win_first = winner < runner-up), at most min(need, hi - e0).
// Lane t evaluates increment t, so a run of up to 64 costs one LDS round trip
// and a ballot instead of one dependent LDS round trip per increment; longer
// runs continue in the next round (the winner is then the same device).
// Returns the (wave-uniform) run length.
template <class SG>
__device__ inline int take_run(const double *G, int e0, int hi, int need, double m2, bool win_first, const SG &sg) {
    const int lim = min(need, hi - e0);
    const int t = sg.sl;
    bool fail = true;
    if (t >= 1 && t < lim) {
        const double x = G[e0 + t + 1] - G[e0 + t];
        fail = !(x < m2 || (x == m2 && win_first));
    }
    const uint64_t nb = sg.bits(t >= 1 && fail);
    return min(nb ? int(__builtin_ctzll(nb)) : SG::S, lim);
}
__device__ inline int take_run(const double *G, int e0, int hi, int need, double m2, bool win_first, int lane) {
    return take_run(G, e0, hi, need, m2, win_first, Wave(lane));
}

// Separable convex allocation by the greedy exchange: start every device at its
// first allowed e, then hand out the remaining R - sum(lo) layers one at a time
// to the device whose next increment G_i[e+1] - G_i[e] is smallest (ties ->
// lowest device index). Optimal because every leaf is convex on its interval.
// The wave is the priority queue: one wave_min per step. Leaves e_i in st0.
__device__ double greedy_alloc(const WaveCtx &w, int M, int R1, int RS, const LeafInfo &li, int lane) {
    int need = (R1 - 1) - li.lo_sum;
    if (li.empty || need < 0 || need > li.cap) return kInf;
    for (int i = lane; i < M; i += 64) {
        const int2 r = w.rng[i];
        const double *G = w.G + int64_t(i) * RS;
        w.st0[i] = r.x;
        w.inc[i] = r.x < r.y ? G[r.x + 1] - G[r.x] : kInf;
    }
    wave_sync();
    // Rounds: the device with the smallest next increment (ties -> lowest index)
    // takes every further increment that still beats the runner-up, so a round
    // equals a run of one-at-a-time greedy steps.
    while (need > 0) {
        double bv = kInf, sv = kInf;
        int bi = 0x7fffffff, si = 0x7fffffff;
        for (int i = lane; i < M; i += 64) {
            const double v = w.inc[i];
            if (v < bv) { sv = bv; si = bi; bv = v; bi = i; }
            else if (v < sv) { sv = v; si = i; }
        }
        const double m = wave_min(bv);
        const int win = wave_imin(bv == m ? bi : 0x7fffffff);
        const int wl = win & 63;
        const double rv = lane == wl ? sv : bv;
        const int ri = lane == wl ? si : bi;
        const double m2 = wave_min(rv);
        const int d2 = wave_imin(rv == m2 ? ri : 0x7fffffff);
        const int t = take_run(w.G + int64_t(win) * RS, w.st0[win], w.rng[win].y, need, m2, win < d2, lane);
        if (lane == wl) {
            const int e = w.st0[win] + t, hi = w.rng[win].y;
            const double *G = w.G + int64_t(win) * RS;
            w.st0[win] = e;
            w.inc[win] = e < hi ? G[e + 1] - G[e] : kInf;
        }
        need -= t;
        wave_sync();
    }
    double S = 0.0;
    for (int i = lane; i < M; i += 64) S += w.G[int64_t(i) * RS + w.st0[i]];
    for (int o = 32; o > 0; o >>= 1) S += __shfl_xor(S, o);
    return S;
}

// Tree min-plus DP over the devices. Leaves: A_i[e] = G[i][e] (masked to +inf
// where H[i][e] > T when use_T). Level l pairs the nodes of level l-1:
// out_p[r] = min_e L[e] + R[r - e] (argmin e -> split, smallest e on ties);
// an unpaired last node passes through. Output node p of level l lives in slot
// p << (l - 1) of `buf` (in place over its left child; buf may be G itself when
// the leaves are not needed again). Returns the root value at r = R (lane-uniform).
// convex: every node is a convex sequence on its finite range rng[slot], so
// e -> L[e] + R[r - e] is convex and its least minimiser is found by binary
// search on f(e + 1) >= f(e) (O(log R) per state); otherwise the O(R) scan.
__device__ double tree_dp(const WaveCtx &w, int M, int R1, int RS, bool use_T, double T, double *buf, int lane,
                          bool convex) {
    if (M == 1) {
        const double g = w.G[R1 - 1];
        return (use_T && !(w.H[R1 - 1] <= T)) ? kInf : g;
    }
    int n = M, l = 0, soff = 0;
    const int npp = R1 <= 64 ? 64 / R1 : 1;  // output nodes per pass
    // R1 > 64: one node per pass, 128 states (two per lane) per chunk. Node p's output overwrites its
    // left child in place, and state r reads the left child only at e <= r, so the chunks run from
    // the highest states down: a chunk never reads what an earlier (higher) chunk wrote.
    const int nch = R1 <= 64 ? 1 : (R1 + 127) >> 7;
    while (n > 1) {
        const int nout = (n + 1) >> 1;
        ++l;
        const double *src = l == 1 ? w.G : buf;
        const int sh = l == 1 ? 0 : l - 2;  // slot shift of this level's inputs
        for (int q = 0; q < ((nout + npp - 1) / npp) * nch; ++q) {
            const int p0 = (q / nch) * npp, r0 = (nch - 1 - q % nch) << 7;
            // each lane: one (node, r) task, or two states of one node when R1 > 64
            double best[2] = {kInf, kInf};
            int be[2] = {0, 0}, pp[2] = {-1, -1}, rr[2] = {0, 0};
            int2 orng[2] = {make_int2(0, -1), make_int2(0, -1)};
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                int p, r;
                if (R1 <= 64) {
                    const int k = lane / R1;
                    p = p0 + k;
                    r = lane - k * R1;
                    if (t > 0 || k >= npp || p >= nout) continue;
                } else {
                    p = p0;
                    r = r0 + lane + 64 * t;
                    if (r >= R1) continue;
                }
                pp[t] = p;
                rr[t] = r;
                const int a = 2 * p, b = 2 * p + 1;
                const int sa = a << sh, sb = b << sh;
                const double *A = src + int64_t(sa) * RS;
                if (b < n) {
                    const double *Bv = src + int64_t(sb) * RS;
                    if (convex) {
                        const int2 ra = w.rng[sa], rb = w.rng[sb];
                        orng[t] = make_int2(ra.x + rb.x, min(ra.y + rb.y, R1 - 1));
                        int lo = max(ra.x, r - rb.y), hi = min(ra.y, r - rb.x);
                        if (lo <= hi) {
                            while (lo < hi) {
                                const int mid = (lo + hi) >> 1;
                                const double f0 = A[mid] + Bv[r - mid], f1 = A[mid + 1] + Bv[r - mid - 1];
                                if (f1 >= f0) hi = mid;
                                else lo = mid + 1;
                            }
                            best[t] = A[lo] + Bv[r - lo];
                            be[t] = lo;
                        }
                    } else {
                        const bool masked = l == 1 && use_T;
                        const double *HA = w.H + int64_t(a) * RS, *HB = w.H + int64_t(b) * RS;
                        // e runs to R1 - 1 on every lane in blocks of 8 (16 LDS reads in
                        // flight before the first use); e > r is masked
                        for (int e0 = 0; e0 < R1; e0 += 8) {
                            double xs[8], ys[8];
#pragma unroll
                            for (int k = 0; k < 8; ++k) {
                                const int ea = min(e0 + k, R1 - 1), eb = max(r - e0 - k, 0);
                                xs[k] = A[ea];
                                ys[k] = Bv[eb];
                                if (masked) {
                                    if (!(HA[ea] <= T)) xs[k] = kInf;
                                    if (!(HB[eb] <= T)) ys[k] = kInf;
                                }
                            }
#pragma unroll
                            for (int k = 0; k < 8; ++k) {
                                const double v = xs[k] + ys[k];
                                if (e0 + k <= r && v < best[t]) { best[t] = v; be[t] = e0 + k; }
                            }
                        }
                    }
                } else {
                    double x = A[r];
                    if (convex) {
                        orng[t] = w.rng[sa];
                        if (r < orng[t].x || r > orng[t].y) x = kInf;
                    } else if (l == 1 && use_T && !(w.H[int64_t(a) * RS + r] <= T)) {
                        x = kInf;
                    }
                    best[t] = x;
                    be[t] = r;
                }
            }
            wave_sync();  // every read of this pass before any write
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                if (pp[t] >= 0) {
                    const int slot = pp[t] << (l - 1);
                    buf[int64_t(slot) * RS + rr[t]] = best[t];
                    w.split[soff + pp[t] * R1 + rr[t]] = uint16_t(be[t]);
                    if (convex && rr[t] == 0) w.rng[slot] = orng[t];
                }
            }
            wave_sync();
        }
        soff += nout * R1;
        n = nout;
    }
    return buf[R1 - 1];
}

// Walk the tree top-down from the root state R: st0[i] = e_i of device i.
__device__ void tree_backtrack(const WaveCtx &w, int M, int R1, int lane) {
    if (M == 1) {
        if (lane == 0) w.st0[0] = R1 - 1;
        wave_sync();
        return;
    }
    // level sizes and split offsets
    int sizes[12];
    int offs[12];
    int L = 0, n = M, soff = 0;
    while (n > 1) {
        const int nout = (n + 1) >> 1;
        sizes[L] = n;  // inputs of level L + 1
        offs[L] = soff;
        soff += nout * R1;
        n = nout;
        ++L;
    }
    int *cur = w.st0, *nxt = w.st1;
    if (lane == 0) cur[0] = R1 - 1;
    wave_sync();
    for (int l = L; l >= 1; --l) {
        const int nin = sizes[l - 1];
        const int nout = (nin + 1) >> 1;
        for (int p = lane; p < nout; p += 64) {
            const int r = cur[p];
            const int e = w.split[offs[l - 1] + p * R1 + r];
            nxt[2 * p] = e;
            if (2 * p + 1 < nin) nxt[2 * p + 1] = r - e;
        }
        wave_sync();
        int *t = cur; cur = nxt; nxt = t;
    }
    if (cur != w.st0) {
        for (int i = lane; i < M; i += 64) w.st0[i] = cur[i];
        wave_sync();
    }
}

// One DP call: leaf ranges / convexity check, then the greedy exchange (convex
// leaves, few layers to hand out) or the tree; leaves the chosen e_i in st0 and
// returns the minimum (+inf when infeasible).
__device__ double dp_call(const WaveCtx &w, int M, int R1, int RS, bool use_T, double T, double *buf, int lane,
                          LeafInfo *li_out = nullptr) {
    if (M > 1) {
        const LeafInfo li = leaf_ranges(w, M, R1, RS, use_T, T, lane, li_out != nullptr);
        if (li_out) *li_out = li;
        wave_sync();
        if (li.convex && (R1 - 1) - li.lo_sum <= 48) return greedy_alloc(w, M, R1, RS, li, lane);
        const double v = tree_dp(w, M, R1, RS, use_T, T, buf, lane, li.convex);
        if (v < kInf) tree_backtrack(w, M, R1, lane);
        return v;
    }
    const double v = tree_dp(w, M, R1, RS, use_T, T, buf, lane, false);
    if (v < kInf) tree_backtrack(w, M, R1, lane);
    return v;
}

struct Inst {
    int inst, m, M, iC, W, R1, RS;
    float invM;
    int64_t co, ro;
    const int32_t *rp;
    double Wd, kc;
};

// Device pass (lane = device): cost / bound / integrality checks, and the
// device's objective entries into LDS. Returns sum_i lb(w_i) on every lane
// and ORs failures into bad.
__device__ int device_pass(const halda_batch &B, const WaveCtx &w, const Inst &I, int lane, int &bad) {
    const int M = I.M;
    const int64_t co = I.co;
    int sumlo = 0;
    for (int i = lane; i < M; i += 64) {
        double cv[6];
        uint8_t ig[6];
#pragma unroll
        for (int b = 0; b < 6; ++b) {
            cv[b] = B.c[co + b * M + i];
            ig[b] = B.integrality[co + b * M + i];
        }
        const double lbw = B.col_lb[co + i], lbn = B.col_lb[co + M + i];
        const double cz = B.c[co + 6 * M + i], lz = B.col_lb[co + 6 * M + i], uz = B.col_ub[co + 6 * M + i];
        const uint8_t iz = B.integrality[co + 6 * M + i];
#pragma unroll
        for (int b = 0; b < 6; ++b) {
            bad |= ig[b] != 1;
            w.cost[6 * i + b] = cv[b];
        }
        bad |= iz != 0 || cz != 0.0 || lz != 0.0 || uz != kInf || lbn < 0.0;
#pragma unroll
        for (int j = 0; j < 4; ++j) bad |= !(cv[2 + j] >= 0.0);
        sumlo += int(ceil(lbw));
        w.cnt[i] = 0;
    }
    if (lane == 0)
        bad |= !(I.kc >= 0.0) || B.integrality[I.co + I.iC] != 0 || B.col_lb[I.co + I.iC] != 0.0 ||
               B.col_ub[I.co + I.iC] != kInf;
    return wave_sum(sumlo);
}

// j = blk * M + i with 0 <= i < M, without an integer division (j < 2^24).
__device__ inline int block_of(int j, int M, float invM) {
    int q = int(float(j) * invM);
    q += (q + 1) * M <= j;
    q -= q * M > j;
    return q;
}

// Cycle row of one device (its last entry is C): busy(i) +- z_i - C <= rhs,
// whose non-w part must equal the device's objective entries. Records the w
// coefficient and rhs. Returns nonzero when the row does not fit.
template <int NZ>
__device__ inline int decode_cycle_row(const WaveCtx &w, const Inst &I, int nnz, double rhs, double vlast, int zc,
                                       double vz, const int (&cols)[NZ], const double (&vals)[NZ]) {
    const int M = I.M;
    const int dev = zc - 6 * M;
    if (vlast != -1.0 || nnz < 2 || dev < 0 || dev >= M || fabs(vz) != 1.0) return 1;
    const double *cst = w.cost + 6 * dev;
    double coef0 = 0.0;
    int seen = 0, rb = 0;  // seen: bitmask of blocks present
#pragma unroll
    for (int k = 0; k < NZ; ++k) {
        if (k < nnz - 2) {
            const int j = cols[k];
            const int blk = block_of(j, M, I.invM);
            if (j >= 6 * M || j - blk * M != dev) rb = 1;
            else if (blk == 0) coef0 = vals[k];
            else {
                rb |= vals[k] != cst[blk];
                seen |= 1 << blk;
            }
        }
    }
    // absent entries must be zero in the objective too
#pragma unroll
    for (int b = 1; b < 6; ++b) rb |= !((seen >> b) & 1) && cst[b] != 0.0;
    if (!rb) {
        const bool first = vz > 0.0;
        w.cyc[4 * dev + (first ? 0 : 1)] = coef0;
        w.cyc[4 * dev + (first ? 2 : 3)] = rhs;
        atomicAdd(&w.cnt[dev], first ? (1 << 8) : (1 << 16));
    }
    return rb;
}

// Capacity / link row of one device: aw w + an n - beta s <= rhs (at most one
// slack column). Records (slack, u, v, K). Returns nonzero when it does not fit.
template <int NZ>
__device__ inline int decode_cap_row(const WaveCtx &w, const Inst &I, int nnz, double rhs, const int (&cols)[NZ],
                                     const double (&vals)[NZ]) {
    int dev = -1, slack = -1, rb = 0;
    double aw = 0.0, an = 0.0, beta = 0.0;
#pragma unroll
    for (int k = 0; k < NZ; ++k) {
        if (k < nnz) {
            const int j = cols[k], blk = block_of(j, I.M, I.invM), i = j - blk * I.M;
            if (j >= 6 * I.M || (dev >= 0 && i != dev)) rb = 1;
            dev = i;
            if (blk == 0) aw = vals[k];
            else if (blk == 1) an = vals[k];
            else if (slack >= 0) rb = 1;
            else { slack = blk - 2; beta = -vals[k]; }
        }
    }
    const double scale = slack >= 0 ? beta : fmax(fabs(aw), fabs(an));
    rb |= !(scale > 0.0) || !(aw == 0.0 || fabs(aw) == scale) || !(an == 0.0 || fabs(an) == scale);
    const int u = aw == 0.0 ? 0 : (aw > 0.0 ? 1 : -1);
    const int v = an == 0.0 ? 0 : (an > 0.0 ? 1 : -1);
    rb |= u * v > 0;  // L-natural convexity: w and n may be coupled only through w - n
    if (rb) return 1;
    const double kk = slack >= 0 ? ceil(-rhs / beta - kSlackEps)
                                 : floor((rhs + kSlackEps * fmax(1.0, fabs(rhs))) / scale);
    if (!(fabs(kk) < 1e8)) return 1;
    const int q = atomicAdd(&w.cnt[dev], 1) & 0xff;
    if (q >= kRows) return 1;
    w.rows[dev * kRows + q] = make_int2((slack + 1) | ((u + 1) << 8) | ((v + 1) << 16), int(kk));
    return 0;
}

// Classify one CSR row by its nonzero pattern and record it for its device.
// Returns nonzero when the row does not fit the HALDA structure.
__device__ inline int decode_row(const WaveCtx &w, const Inst &I, int nnz, double rhs, double rlb,
                                 const int (&cols)[kMaxRowNnz], const double (&vals)[kMaxRowNnz]) {
    if (rlb != -kInf || nnz < 1 || nnz > kMaxRowNnz || !(fabs(rhs) < 1e300)) return 1;
    int last = -1, zc = -1;
    double vlast = 0.0, vz = 0.0;
#pragma unroll
    for (int k = 0; k < kMaxRowNnz; ++k) {
        if (k == nnz - 1) { last = cols[k]; vlast = vals[k]; }
        if (k == nnz - 2) { zc = cols[k]; vz = vals[k]; }
    }
    if (last == I.iC) return decode_cycle_row<kMaxRowNnz>(w, I, nnz, rhs, vlast, zc, vz, cols, vals);
    return decode_cap_row<kMaxRowNnz>(w, I, nnz, rhs, cols, vals);
}

// Row pass: lane-strided rows, two rows per lane per step; the next step's row
// pointers / bounds are loaded together with this step's entries (one global
// round trip per step).
__device__ int row_pass(const halda_batch &B, const WaveCtx &w, const Inst &I, int lane) {
    const int nr = I.m - 1;
    int bad = 0;
    int rs[2], re[2];
    double rhs[2], rlb[2];
    auto meta = [&](int r0) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int r = r0 + 64 * h + lane;
            const bool in = r < nr;
            rs[h] = in ? I.rp[r] : 0;
            re[h] = in ? I.rp[r + 1] : 0;
            rhs[h] = in ? B.row_ub[I.ro + r] : 0.0;
            rlb[h] = in ? B.row_lb[I.ro + r] : -kInf;
        }
    };
    meta(0);
    for (int r0 = 0; r0 < nr; r0 += 128) {
        int cols[2][kMaxRowNnz];
        double vals[2][kMaxRowNnz];
        int nnz[2];
        double hr[2], lr[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            nnz[h] = re[h] - rs[h];
            hr[h] = rhs[h];
            lr[h] = rlb[h];
#pragma unroll
            for (int k = 0; k < kMaxRowNnz; ++k) {
                const bool in = k < nnz[h];
                cols[h][k] = in ? B.col_idx[rs[h] + k] : -1;
                vals[h][k] = in ? B.val[rs[h] + k] : 0.0;
            }
        }
        if (r0 + 128 < nr) meta(r0 + 128);
#pragma unroll
        for (int h = 0; h < 2; ++h)
            if (r0 + 64 * h + lane < nr) bad |= decode_row(w, I, nnz[h], hr[h], lr[h], cols[h], vals[h]);
    }
    return bad;
}

// Capacity-row staging of the k = 1 decode (decode_k1).
constexpr int kCapNnz = 3;     // widest capacity / link row (w, n, one slack)
constexpr int kCapSlots = 4;   // capacity rows per lane: up to 256 rows
constexpr int kCycSlots = 2;   // cycle rows per lane: 2M <= 128

// Per device: one row of each cycle kind, <= 2 pure rows, and the rows of one
// slack share their (u, v) pattern.
__device__ int check_rows(const WaveCtx &w, int M, int lane) {
    int bad = 0;
    for (int i = lane; i < M; i += 64) {
        const int c = w.cnt[i], nr = min(c & 0xff, kRows);
        bad |= (c & 0xff) > kRows || ((c >> 8) & 0xff) != 1 || ((c >> 16) & 0xff) != 1;
        int pure = 0;
        for (int q = 0; q < nr; ++q) {
            const int x = w.rows[i * kRows + q].x, kind = (x & 0xff) - 1;
            pure += kind < 0;
            for (int q2 = 0; q2 < q; ++q2) {
                const int x2 = w.rows[i * kRows + q2].x;
                bad |= kind >= 0 && (x2 & 0xff) == (x & 0xff) && (x2 >> 8) != (x >> 8);
            }
        }
        bad |= pure > 2;
    }
    return bad;
}

// One table entry e of device i, continuing the chain state (n, have).
template <class Rec>
__device__ inline void table_entry(const Rec &d, const WaveCtx &w, const Inst &I, int i, int e, int &n, bool &have) {
    const int wl = rec_wlo(d) + e;
    int s[4];
    double g = kInf, h = kInf;
    bool ok = false;
    if (wl <= rec_whi(d)) ok = have ? split_step(d, wl, n, g, n, s) : split_full(d, wl, g, n, s);
    if (ok && I.kc > 0.0) h = fmax(0.0, least_cycle(d, wl, n, s));
    have = ok;
    w.G[i * I.RS + e] = ok ? g : kInf;
    if (I.kc > 0.0) w.H[i * I.RS + e] = h;
}

// Device records of an instance decoded from its CSR (load_dev).
struct CsrSrc {
    using Rec = Dev;
    const halda_batch *B;
    int64_t co;
    int M;
    double Wd;
    __device__ inline void load(Dev &d, const WaveCtx &w, int i) const { load_dev(d, *B, w, co, M, i, Wd); }
};

// Table pass (lane = device): G[i][e] (and H[i][e] for k > 1), w = lb + e, one
// incremental chain per device (split_step reuses the previous argmin).
// Fleets of at most 32 devices spread each device's chain over P = 64 / M lanes
// (each starts its stretch of e with a full split search): the least minimiser
// n*(w) is the same either way, so G and H are too.
// src.load runs on every lane (index clamped to a valid device) so that a source may shuffle
// records between lanes.
template <int S = 64, class Src>
__device__ void table_pass(const Src &src, const WaveCtx &w, const Inst &I, int lane) {
    if (I.M <= S / 2) {
        const int P = S / I.M, chunk = (I.R1 + P - 1) / P;
        const int i = lane / P, p = lane - i * P;
        typename Src::Rec d;
        src.load(d, w, min(i, I.M - 1));
        if (i < I.M) {
            int n = 0;
            bool have = false;
            const int e1 = min(I.R1, (p + 1) * chunk);
            for (int e = p * chunk; e < e1; ++e) table_entry(d, w, I, i, e, n, have);
        }
        return;
    }
    for (int i0 = 0; i0 < I.M; i0 += S) {
        const int i = i0 + lane;
        typename Src::Rec d;
        src.load(d, w, min(i, I.M - 1));
        if (i < I.M) {
            int n = 0;
            bool have = false;
            for (int e = 0; e < I.R1; ++e) table_entry(d, w, I, i, e, n, have);
        }
    }
}

// k > 1: incremental threshold scan (lane = device, M <= 64). When every leaf
// is convex on its finite range and its least cycle time H_i(e) is
// nondecreasing in e, the mask H_i(e) <= T is a cap e_i <= cap_i(T), and the
// capped problem S(T) is a separable convex allocation with box constraints:
// an allocation is optimal iff its largest taken increment is no larger than
// its smallest available one. Raising T past the next candidate value raises
// ONE device's cap by one, which makes at most one new increment available, so
// the optimum of the next T is the current one plus at most one exchange (take
// the new increment, drop the largest taken one when the new one is smaller).
// The scan thus costs a few wave reductions per candidate T instead of a full
// DP pass (leaf scan + greedy / tree + backtrack). Candidates are visited in
// ascending T (a merge of the devices' sorted H rows) with the same pruning as
// the pass-per-candidate scan: stop once (k-1) T + S(inf) >= best. Returns
// false (caller runs the general scan) when a leaf is not convex / monotone.
// On success st0 holds the allocation (table indices e_i).
template <class SG>
__device__ bool kc_scan_incremental(const WaveCtx &w, const Inst &I, const SG &sg, double s_inf, double best0,
                                    int64_t &nodes, const LeafInfo &li0) {
    const int M = I.M, R1 = I.R1, RS = I.RS;
    const double kc = I.kc;
    const int lane = sg.sl;  // device index within the problem
    if (M > SG::S || M < 2 || !li0.convex || !li0.mono || li0.empty) return false;
    HALDA_KSTAMP(3);
    const bool act = lane < M;
    const double *G = w.G + int64_t(act ? lane : 0) * RS, *H = w.H + int64_t(act ? lane : 0) * RS;
    const int lo = act ? li0.my_lo : 0, hi = act ? li0.my_hi : -1;
    const int need_total = (R1 - 1) - li0.lo_sum;
    if (need_total < 0 || need_total > li0.cap) return false;
    // start at T0 = max_i H_i(lo_i): every device can sit at its first allowed e
    double T = sg.max_f64(act ? H[lo] : -kInf);
    int cap = lo;
    if (act)
        while (cap < hi && H[cap + 1] <= T) ++cap;
    // optimal capped allocation at T0 (greedy: every cap filled from lo, then the smallest increments)
    int e = lo;
    int need = need_total;
    {
        const int avail = sg.sum_i(act ? cap - lo : 0);
        if (avail <= need) {  // take everything allowed (incomplete when avail < need)
            e = cap;
            need -= avail;
        } else {
            while (need > 0) {  // rounds: the smallest next increment wins and keeps every one beating the runner-up
                const double nx = act && e < cap ? G[e + 1] - G[e] : kInf;
                const double bv = sg.min_f64(nx);
                const int win = sg.lowest(nx == bv);
                const double rv = lane == win ? kInf : nx;
                const double m2 = sg.min_f64(rv);
                const int d2 = sg.lowest(rv == m2);
                const int t = take_run(w.G + int64_t(win) * RS, sg.bcast(e, win), sg.bcast(cap, win), need, m2, win < d2,
                                       sg);
                if (lane == win) e += t;
                need -= t;
            }
        }
    }
    double S = sg.sum_f64(act ? G[e] : 0.0);
    HALDA_KSTAMP(4);
    double best = best0;
    int bestE = -1;
    int64_t events = 0;
    // Only "useful" cap openings change the optimum: device i must sit at its cap (e_i == cap_i; a
    // device below its cap already declined a unit no worse than its next) and the unit its next cap
    // opens must be needed (allocation incomplete) or beat the largest taken unit lam. lam only
    // decreases, so a device that is not useful now never becomes useful except the one that just
    // took a unit; the scan therefore jumps T straight to the next useful opening and costs one
    // reduction per exchange instead of one per candidate T.
    double hn = act && cap < hi ? H[cap + 1] : kInf;   // H of this device's next cap
    double gn = act && cap < hi ? G[cap + 1] - G[cap] : kInf;  // the unit it opens (cap -> cap + 1)
    double lt = act && e > lo ? G[e] - G[e - 1] : -kInf;  // its last taken unit
    double lam = -kInf;
    int lj = -1;
    if (need == 0) {
        lam = sg.max_f64(lt);
        lj = sg.highest(lt == lam);
        if (kc * T + S < best) {
            best = kc * T + S;
            bestE = e;
        }
    }
    while (true) {
        const bool useful = act && e == cap && cap < hi && (need > 0 || gn < lam);
        const double cand = useful ? hn : kInf;
        const double Tn = sg.min_f64(cand);
        if (!(Tn < kInf) || !(kc * Tn + s_inf < best)) break;
        const int li = sg.lowest(cand == Tn);
        ++events;
        const double d = sg.bcast(gn, li);
        const bool swap = need == 0;  // else: fill
        const int ljo = lj;
        S += swap ? d - lam : d;
        if (!swap) --need;
        // li takes the unit its new cap opens; ljo gives back its largest taken unit (li == ljo only
        // through the convexity tolerance: then in that order). All LDS reads in one round trip.
        const bool is_li = lane == li, is_lj = swap && lane == ljo;
        if (is_li || is_lj) {
            const int ncap = is_li ? e + 1 : cap;
            const int ne = is_li ? (is_lj ? e : e + 1) : e - 1;
            const int a = min(ncap + 1, hi), b = max(ne - 1, 0);
            const double Gn1 = G[a], Gn0 = G[ncap], Hn1 = H[a], Ge = G[ne], Gm = G[b];
            if (is_li) {
                cap = ncap;
                hn = cap < hi ? Hn1 : kInf;
                gn = cap < hi ? Gn1 - Gn0 : kInf;
            }
            e = ne;
            lt = is_lj ? (e > lo ? Ge - Gm : -kInf) : Ge - Gm;
        }
        if (need == 0) {
            lam = sg.max_f64(lt);
            lj = sg.highest(lt == lam);
        }
        T = Tn;
        if (need == 0 && kc * T + S < best) {
            best = kc * T + S;
            bestE = e;
        }
    }
    nodes += events;
    HALDA_KSTAMP(5);
    if (bestE >= 0) {  // a capped optimum beat the unconstrained allocation's own T
        if (act) w.st0[lane] = bestE;
    }
    wave_sync();
    return true;
}

// k > 1 for fleets of at most 64 devices with convex leaves and nondecreasing cycle times (every
// instance the reference builds): lane = device, the leaf scan and the phase-0 greedy exchange in
// registers (the same choices as leaf_ranges + greedy_alloc: smallest increment first, ties to the
// lowest device, runs taken while they beat the runner-up), then the incremental threshold scan.
// Returns 1 solved (st0 = allocation), 0 infeasible, -1 not applicable (the table DP below runs).
template <class SG>
__device__ int dp_pass_lanes(const WaveCtx &w, const Inst &I, const SG &sg, int64_t &nodes) {
    const int M = I.M, R1 = I.R1, RS = I.RS;
    const int lane = sg.sl;
    const bool act = lane < M;
    const double *G = w.G + int64_t(act ? lane : 0) * RS, *H = w.H + int64_t(act ? lane : 0) * RS;
    int lo = R1, hi = -1, cnt = 0;
    bool ok = true, mono = true;
    double prev = kInf, dprev = -kInf, hprev = -kInf;
    if (act)
        for (int e = 0; e < R1; ++e) {
            const double g = G[e], h = H[e];
            if (g < kInf) {
                if (cnt > 0) {
                    const double d = g - prev;
                    ok = ok && (hi == e - 1) && d >= dprev - 1e-12 * fmax(1.0, fabs(g));
                    dprev = d;
                }
                mono = mono && h >= hprev;
                hprev = h;
                lo = min(lo, e);
                hi = e;
                prev = g;
                ++cnt;
            }
        }
    if (sg.any(act && (!ok || !mono))) return -1;
    if (sg.any(act && cnt == 0)) return 0;
    LeafInfo li;
    li.convex = true;
    li.mono = true;
    li.empty = false;
    li.lo_sum = sg.sum_i(act ? lo : 0);
    li.cap = sg.sum_i(act ? hi - lo : 0);
    li.my_lo = act ? lo : 0;
    li.my_hi = act ? hi : -1;
    int need = (R1 - 1) - li.lo_sum;
    if (need < 0 || need > li.cap) return 0;
    // phase 0: unconstrained greedy exchange (rounds: the smallest next increment wins and keeps
    // every one still beating the runner-up)
    int e = act ? lo : 0;
    double inc = act && e < hi ? G[e + 1] - G[e] : kInf;
    while (need > 0) {
        const double bv = sg.min_f64(inc);
        const int win = sg.lowest(inc == bv);
        const double rv = lane == win ? kInf : inc;
        const double m2 = sg.min_f64(rv);
        const int d2 = sg.lowest(rv == m2);
        const int t = take_run(w.G + int64_t(win) * RS, sg.bcast(e, win), sg.bcast(hi, win), need, m2, win < d2, sg);
        if (lane == win) {
            e += t;
            inc = e < hi ? G[e + 1] - G[e] : kInf;
        }
        need -= t;
    }
    const double s_inf = sg.sum_f64(act ? G[e] : 0.0);
    const double hmax = sg.max_f64(act ? fmax(0.0, H[e]) : 0.0);
    if (act) w.st0[lane] = e;
    nodes = 1;
    kc_scan_incremental(w, I, sg, s_inf, I.kc * hmax + s_inf, nodes, li);
    wave_sync();
    return 1;
}

// DP pass; k > 1: ascending threshold scan with bound pruning. One tree_dp call
// site: phase 0 = unconstrained, 1 = threshold scan, 2 = final re-run. Leaves the
// chosen e_i in st0; returns false when infeasible.
__device__ bool dp_pass(const WaveCtx &w, const Inst &I, int lane, int64_t &nodes) {
#ifndef HALDA_NO_LANE_DP
    if (I.kc > 0.0 && I.M >= 2 && I.M <= 64) {
        const int r = dp_pass_lanes(w, I, Wave(lane), nodes);
        if (r >= 0) return r == 1;
    }
#endif
    const int M = I.M, R1 = I.R1, RS = I.RS;
    const double kc = I.kc;
    double *buf = kc > 0.0 ? w.work : w.G;
    int phase = 0;
    bool use_T = false;
    double T = 0.0, s_inf = kInf, best = kInf, bestT = kInf, tprev = -1.0, tlo = 0.0;
    nodes = 0;
    LeafInfo li0 = {};
    while (true) {
        const double st = dp_call(w, M, R1, RS, use_T, T, buf, lane, phase == 0 && kc > 0.0 ? &li0 : nullptr);
        ++nodes;
        if (phase == 2) break;
        if (phase == 0) {
            HALDA_KSTAMP(1);
            s_inf = st;
            if (!(st < kInf)) return false;
            if (!(kc > 0.0)) break;  // k = 1: the allocation of this pass is final
            double hmax = 0.0;
            for (int i = lane; i < M; i += 64) hmax = fmax(hmax, w.H[i * RS + w.st0[i]]);
            hmax = wave_max(hmax);
            best = kc * hmax + s_inf;
            phase = 1;
            HALDA_KSTAMP(2);
            // convex leaves with monotone cycle times: one exchange per candidate T
            if (kc_scan_incremental(w, I, Wave(lane), s_inf, best, nodes, li0)) return true;
            for (int i = lane; i < M; i += 64) {
                double mn = kInf;
                for (int e = 0; e < R1; ++e)
                    if (w.G[i * RS + e] < kInf) mn = fmin(mn, w.H[i * RS + e]);
                tlo = fmax(tlo, mn);  // every assignment has max_i H_i >= max_i min_e H[i][e]
            }
            tlo = wave_max(tlo);
        } else if (st < kInf && kc * T + st < best) {
            best = kc * T + st;
            bestT = T;
        }
        if (phase == 1) {
            if (use_T) tprev = T;
            double t = kInf;
            for (int i = lane; i < M; i += 64)
                for (int e = 0; e < R1; ++e) {
                    const double h = w.H[i * RS + e];
                    if (w.G[i * RS + e] < kInf && h >= tlo && h > tprev) t = fmin(t, h);
                }
            t = wave_min(t);
            if (t < kInf && kc * t + s_inf < best) {
                use_T = true;
                T = t;
                continue;
            }
            if (!use_T && !(bestT < kInf)) break;  // no scan pass ran: the phase-0 allocation is final
            phase = 2;
            use_T = bestT < kInf;
            T = bestT;
        }
    }
    return true;
}

// Output pass (lane = device): x = (w, n, least slacks, stall z, cycle time C), obj_lin.
__device__ void output_pass(const halda_batch &B, const halda_result &Rz, const WaveCtx &w, const Inst &I, int lane,
                            int64_t nodes) {
    const int M = I.M;
    double hmax = 0.0;
    double *x = Rz.x + I.co;
    for (int i = lane; i < M; i += 64) {
        Dev d;
        load_dev(d, B, w, I.co, I.M, i, I.Wd);
        const int wl = d.wlo + w.st0[i];
        double g = 0.0, P, Q;
        int n = 0, s[4] = {0, 0, 0, 0};
        split_full(d, wl, g, n, s);
        dev_cycle(d, wl, n, s, P, Q);
        x[i] = double(wl);
        x[M + i] = double(n);
        x[2 * M + i] = double(s[0]);
        x[3 * M + i] = double(s[1]);
        x[4 * M + i] = double(s[2]);
        x[5 * M + i] = double(s[3]);
        x[6 * M + i] = Q > P ? 0.5 * (Q - P) : 0.0;
        w.cyc[4 * i] = g;  // per-device cost scratch for the ordered sum below
        hmax = fmax(hmax, Q >= P ? 0.5 * (P + Q) : P);
    }
    hmax = wave_max(hmax);
    wave_sync();
    if (lane == 0) {
        double gsum = 0.0;
        for (int i = 0; i < M; ++i) gsum = gsum + w.cyc[4 * i];
        const double obj = gsum + I.kc * hmax;
        x[I.iC] = hmax;
        Rz.status[I.inst] = HALDA_STATUS_OPTIMAL;
        Rz.obj_lin[I.inst] = obj;
        Rz.dual_bound[I.inst] = obj;
        Rz.gap[I.inst] = 0.0;
        Rz.nodes[I.inst] = nodes;
    }
    wave_sync();
}


#ifndef HALDA_SOLVE_WAVES_PER_SIMD
#define HALDA_SOLVE_WAVES_PER_SIMD 2  // occupancy target of the solve kernel (register budget)
#endif

// kGlobal = false: the slice lives in LDS (one wave per 64-thread workgroup). Instances whose shape
// does not fit this launch's slice (M > mmax, R + 1 > r1max or M * RS > its table) are re-tagged
// CLS_BIG for the global-table launch that follows (only launched when the batch's shape summary
// exceeds the LDS budget). kGlobal = true: the same code on a per-wave slice of global scratch
// (gtab + blockIdx.x * gstride bytes), sized from the full shape summary, no size limit but HBM.
template <bool kGlobal>
__device__ inline void solve_general(halda_batch B, halda_result Rz, uint8_t *cls, int mmax, int r1max, int tab,
                                     int tab_kc, const int *hb_flag, int launch_id, int gated, int want,
                                     unsigned char *slice_base) {
    const int lane = threadIdx.x;
    // gated: no k > 1 or wide instance in the batch; only k = 1 hand-backs (flagged) can be here
    if (gated && __hip_atomic_load(hb_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != launch_id) return;
    const Slice sl = make_slice(mmax, r1max, tab, tab_kc);
    unsigned char *base = slice_base;
    WaveCtx w;
    w.rows = reinterpret_cast<int2 *>(base + sl.rows);
    w.cyc = reinterpret_cast<double *>(base + sl.cyc);
    w.cost = reinterpret_cast<double *>(base + sl.cost);
    w.cnt = reinterpret_cast<int *>(base + sl.cnt);
    w.st0 = reinterpret_cast<int *>(base + sl.st0);
    w.st1 = reinterpret_cast<int *>(base + sl.st1);
    w.rng = reinterpret_cast<int2 *>(base + sl.rng);
    w.inc = reinterpret_cast<double *>(base + sl.inc);
    w.G = reinterpret_cast<double *>(base + sl.G);
    w.H = reinterpret_cast<double *>(base + sl.H);
    w.work = reinterpret_cast<double *>(base + sl.work);
    w.split = reinterpret_cast<uint16_t *>(base + sl.split);

    // this wave owns instances blockIdx.x + j * gridDim.x; a 64-wide window of
    // them is screened by one ballot over the verdict bytes
    const int S = gridDim.x;
    for (int64_t base_i = blockIdx.x; base_i < B.n_inst; base_i += int64_t(64) * S) {
        const int64_t mine = base_i + int64_t(lane) * S;
        const bool open = mine < B.n_inst && cls[mine] == want;
        uint64_t todo = __ballot(open);
        while (todo) {
            const int bit = __builtin_ctzll(todo);
            todo &= todo - 1;
            Inst I;
            I.inst = int(base_i + int64_t(bit) * S);
            const int N = B.n_cols[I.inst];
            I.m = B.n_rows[I.inst];
            I.M = (N - 1) / 7;
            I.iC = 7 * I.M;
            I.invM = 1.0f / float(I.M);
            I.co = B.col_off[I.inst];
            I.ro = B.row_off[I.inst];
            I.rp = B.row_ptr + B.csr_off[I.inst];
            I.Wd = B.row_ub[I.ro + I.m - 1];
            I.W = int(I.Wd);
            I.kc = B.c[I.co + I.iC];
            if (!kGlobal && I.M > mmax) {  // wider than this slice: the global-table launch
                if (lane == 0) cls[I.inst] = CLS_BIG;
                continue;
            }
            HALDA_STAMP(0);

            int bad = 0;
            const int sumlo = device_pass(B, w, I, lane, bad);
            I.R1 = I.W - sumlo + 1;
            I.RS = odd_stride(I.R1);
            wave_sync();
            if (!kGlobal && (I.R1 > r1max || int64_t(I.M) * I.RS > (I.kc > 0.0 ? tab_kc : tab))) {
                if (lane == 0) cls[I.inst] = CLS_BIG;  // tables beyond this slice: the global-table launch
                continue;
            }
            HALDA_GSTAMP(1);
            bad |= row_pass(B, w, I, lane);
            wave_sync();
            HALDA_GSTAMP(2);
            bad |= check_rows(w, I.M, lane);
            if (wave_or(bad)) {
                if (lane == 0) write_done(Rz, I.inst, HALDA_STATUS_UNSUPPORTED, 0);
                continue;
            }
            HALDA_GSTAMP(3);
            table_pass(CsrSrc{&B, I.co, I.M, I.Wd}, w, I, lane);
            wave_sync();
            HALDA_GSTAMP(4);
            int64_t nodes = 0;
            if (!dp_pass(w, I, lane, nodes)) {
                if (lane == 0) write_done(Rz, I.inst, HALDA_STATUS_INFEASIBLE, nodes);
                continue;
            }
            HALDA_GSTAMP(5);
            output_pass(B, Rz, w, I, lane, nodes);
            HALDA_STAMP(6);
        }
    }
}

__global__ __launch_bounds__(64, HALDA_SOLVE_WAVES_PER_SIMD) void halda_solve_kernel(
    halda_batch B, halda_result Rz, uint8_t *cls, int mmax, int r1max, int tab, int tab_kc, const int *hb_flag,
    int launch_id, int gated, int want) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    solve_general<false>(B, Rz, cls, mmax, r1max, tab, tab_kc, hb_flag, launch_id, gated, want, smem);
}

// Global-table variant: instances the LDS launches re-tagged CLS_BIG (and, in a batch whose summary
// exceeds the LDS budget, nothing else).
__global__ __launch_bounds__(64, HALDA_SOLVE_WAVES_PER_SIMD) void halda_solve_big_kernel(
    halda_batch B, halda_result Rz, uint8_t *cls, int mmax, int r1max, int tab, int tab_kc, unsigned char *gtab,
    int64_t gstride) {
    solve_general<true>(B, Rz, cls, mmax, r1max, tab, tab_kc, nullptr, 0, 0, CLS_BIG,
                        gtab + int64_t(blockIdx.x) * gstride);
}

// ---------------------------------------------------------------- k = 1 fast path
// c[C] == 0 and M <= 64 (every feasible C3 instance): the cycle rows never bind,
// the problem is min sum_i G_i(e_i) s.t. sum e_i = R with G_i convex, and the
// greedy exchange is exact. No tables: lane i holds device i's record in
// registers and only G_i(0), G_i(1). Each round the device with the smallest
// next increment (ties -> lowest index) wins; the whole wave then evaluates the
// winner's G at its next 64 layer counts in parallel (its record broadcast from
// the winner lane through readlane), and the winner keeps every increment that
// still beats the runner-up's -- one round usually places all R layers, where
// the table path evaluates M x (R + 1) entries. The convexity the exchange
// relies on is re-checked on every evaluated window (same 1e-12 tolerance as
// leaf_ranges); an instance whose leaves do not start at e = 0 or fail the
// check is handed to the general kernel (cls = CLS_GEN), never approximated.

// LDS slice of one k = 1 wave: capacity-row records, per-device row counters
// and a staging buffer for one coalesced CSR segment (kStage entries: col_idx
// then val). The generic decode (hand-back of a CSR in another row order) keeps
// its cyc / cost records in the staging buffer instead.
constexpr int kStage = 512;
constexpr int kStageColBytes = kStage * 4 + 32;  // 16-B chunks from the segment start rounded down
constexpr int kStageValBytes = kStage * 8 + 32;

struct K1Slice {
    int64_t rows, cnt, stage, cyc, cost, total;
};

__host__ __device__ inline K1Slice make_k1_slice(int mmax) {
    K1Slice s;
    int64_t o = 0;
    s.rows = o;  o = align16(o + int64_t(mmax) * kRows * 8);
    s.cnt = o;   o = align16(o + int64_t(mmax) * 4);
    s.stage = o;
    const int64_t st = kStageColBytes + kStageValBytes, rec = int64_t(mmax) * (4 + 6) * 8;
    o = align16(o + (st > rec ? st : rec));
    s.cyc = s.stage;
    s.cost = s.stage + int64_t(mmax) * 4 * 8;
    s.total = o;
    return s;
}

__device__ inline Dev bcast_dev(const Dev &d, int src) {
    Dev o;
    o.cw = bcast(d.cw, src); o.cn = bcast(d.cn, src);
    o.cs0 = bcast(d.cs0, src); o.cs1 = bcast(d.cs1, src); o.cs2 = bcast(d.cs2, src); o.cs3 = bcast(d.cs3, src);
    o.r1w = bcast(d.r1w, src); o.r2w = bcast(d.r2w, src); o.rhs1 = bcast(d.rhs1, src); o.rhs2 = bcast(d.rhs2, src);
    o.wlo = bcast(d.wlo, src); o.whi = bcast(d.whi, src); o.nlo = bcast(d.nlo, src); o.nhi = bcast(d.nhi, src);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        o.slo[j] = bcast(d.slo[j], src); o.shi[j] = bcast(d.shi[j], src);
        o.us[j] = bcast(d.us[j], src); o.vs[j] = bcast(d.vs[j], src); o.Ks[j] = bcast(d.Ks[j], src);
    }
#pragma unroll
    for (int f = 0; f < 2; ++f) {
        o.uf[f] = bcast(d.uf[f], src); o.vf[f] = bcast(d.vf[f], src); o.Kf[f] = bcast(d.Kf[f], src);
    }
    return o;
}


enum { K1_OK = 0, K1_INFEASIBLE = 1, K1_FALLBACK = 2 };

// A device record as the k = 1 greedy sees it: the full Dev (CSR decode) or a compact record
// expanded on use (fused sweep); bcast(src) = lane src's record on every lane.
struct FullRec {
    Dev d;
    __device__ inline Dev dev() const { return d; }
    __device__ inline const Dev &core() const { return d; }
    template <class SG>
    __device__ inline FullRec bcast(const SG &, int src) const {
        static_assert(SG::S == 64, "the CSR k = 1 path runs one problem per wave");
        return FullRec{bcast_dev(d, src)};
    }
};

// Greedy exchange over lazily evaluated convex leaves (lane = device, M <= 64).
// On K1_OK, e holds the device's extra layers.
// gE / nE: the device's G(e) and its least minimiser n at the returned e -- split_full's values at
// w = lb + e, so the caller's output needs no split of its own.
template <class Rec, class SG>
__device__ int k1_alloc(const Rec &rec, int M, int R, const SG &sg, int &e, int &rounds, double &gE, int &nE) {
    const int lane = sg.sl;  // device index within the problem
    const auto &d = rec.core();  // Dev, or the compact record with its specialised split
    const bool act = lane < M;
    double g0 = kInf, g1 = kInf;
    int n0 = 0, n1 = 0, s[4];
    bool ok0 = false, ok1 = false;
    if (act) {
        // both splits evaluated unconditionally (independent: they interleave), used only where valid
        const int wlo = rec_wlo(d), whi = rec_whi(d);
        double ga, gb;
        int na, nb, sb[4];
        const bool fa = split_first(d, wlo, ga, na, s);
        const bool fb = split_full(d, wlo + 1, gb, nb, sb);
        ok0 = wlo <= whi && fa;
        ok1 = ok0 && wlo + 1 <= whi && fb;
        g0 = ok0 ? ga : g0;
        n0 = ok0 ? na : n0;
        g1 = ok1 ? gb : g1;
        n1 = ok1 ? nb : n1;
    }
    e = 0;
    gE = g0;
    nE = n0;
    // every leaf must start at e = 0 (a later start is legal but rare: general kernel)
    if (sg.bits(act && !ok0)) return K1_FALLBACK;
    double gn = ok1 ? g1 : kInf;               // G(e + 1)
    int nN = n1;                               // its n
    double inc = ok1 ? g1 - g0 : kInf;        // G(e + 1) - G(e)
    double dprev = -kInf;                      // last taken increment (convexity check)
    int need = R;
    rounds = 0;
    while (need > 0) {
        ++rounds;
        const double bv = sg.min_f64(act ? inc : kInf);
        if (!(bv < kInf)) return K1_INFEASIBLE;  // no device can take another layer
        const int win = sg.lowest(act && inc == bv);
        const double rv = act && lane != win ? inc : kInf;
        const double m2 = sg.min_f64(rv);
        const int d2 = sg.lowest(act && lane != win && rv == m2);
        const int ew = sg.bcast(e, win), nNw = sg.bcast(nN, win);
        const double gnw = sg.bcast(gn, win);
        // the winner takes its next increment bv; lane t evaluates G_win(ew + 2 + t)
        int take = 1;
        // convexity against the winner's last taken increment (none in the first round: -inf)
        bool bad = rounds > 1 && bv < sg.bcast(dprev, win) - 1e-12 * fmax(1.0, fabs(gnw));
        double Gt = kInf, dt = kInf;
        int nt = 0;
        if (need > 1) {
            const auto dw = rec.bcast(sg, win).core();
            const int wl = rec_wlo(dw) + ew + 2 + lane;
            double g = kInf;
            if (wl <= rec_whi(dw) && split_full(dw, wl, g, nt, s)) Gt = g;
            // shuffles on the full wave first (a bpermute under a lane-0-off mask would read 0 there)
            const double up = sg.up1(Gt);
            const double prev = lane == 0 ? gnw : up;
            dt = Gt - prev;  // increment ew + 1 + lane -> ew + 2 + lane
            const double dup = sg.up1(dt);
            const double dlast = lane == 0 ? bv : dup;
            const bool fin = Gt < kInf && prev < kInf;
            const bool beats = fin && (dt < m2 || (dt == m2 && win < d2));
            const uint64_t nb = sg.bits(!beats);
            const int run = nb ? __builtin_ctzll(nb) : SG::S;  // increments after the first that still win
            take = min(min(1 + run, need), SG::S);
            // convexity over the increments taken and the next one (they decide the exchange)
            bad = bad || sg.bits(fin && lane < take && dt < dlast - 1e-12 * fmax(1.0, fabs(Gt))) != 0;
        }
        if (bad) return K1_FALLBACK;
        // winner's new state: e = ew + take; G(e) from the evaluated window, and G(e + 1) / the last
        // increment for the next round only when there is one (need > take; uniform)
        const double gcur = take == 1 ? gnw : sg.bcast(Gt, take - 2);
        const int ncur = take == 1 ? nNw : sg.bcast(nt, take - 2);
        if (lane == win) {
            e = ew + take;
            gE = gcur;
            nE = ncur;
        }
        if (need > take) {  // then need > 1: the window was evaluated
            const double gnext = sg.bcast(Gt, take - 1);
            const int nnext = sg.bcast(nt, take - 1);
            const double tlast = take == 1 ? bv : sg.bcast(dt, take - 2);
            if (lane == win) {
                gn = gnext;
                nN = nnext;
                inc = gnext < kInf ? gnext - gcur : kInf;
                dprev = tlast;
            }
        }
        need -= take;
    }
    return K1_OK;
}

#ifndef HALDA_K1_WAVES_PER_SIMD
#define HALDA_K1_WAVES_PER_SIMD 4  // occupancy target of the k = 1 kernel (register budget)
#endif

// LDS-DMA staging (global_load_lds_dwordx4): bytes [p, p + nbytes) land in dst
// as lane-linear 16-B chunks from p rounded down to 16 B (each wave
// instruction fills 1 KiB); returns p's byte offset in dst. No VGPR holds the
// data; stage_wait() retires the copies before the LDS is read. Chunks may read
// up to 15 B past the range (the caller guarantees they are in the array).
__device__ inline void glds16(const void *g, void *lds) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)g,
                                     (__attribute__((address_space(3))) void *)lds, 16, 0, 0);
}

__device__ inline int stage_lds(const void *p, int nbytes, unsigned char *dst, int lane) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p), a0 = a & ~uintptr_t(15);
    const int chunks = int((a + uintptr_t(nbytes) - a0 + 15) >> 4);
    for (int c0 = 0; c0 < chunks; c0 += 64)
        if (c0 + lane < chunks) glds16(reinterpret_cast<const void *>(a0 + 16 * uintptr_t(c0 + lane)), dst + 16 * c0);
    return int(a - a0);
}

__device__ inline void stage_wait() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
}

__device__ inline double shfl_f64(double v, int src) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = __shfl(int(uint32_t(u)), src), hi = __shfl(int(uint32_t(u >> 32)), src);
    return __builtin_bit_cast(double, (uint64_t(hi) << 32) | lo);
}

// k = 1 (and W = M) by an exact min-plus DP over the devices, for any leaf shape (lane = r, R + 1 <=
// kDpLanes): the register sweep's own fallback for what the greedy exchange does not take (a leaf
// that is not convex within its tolerance, or that does not start at lb), so that the register
// launch needs no table launch behind it. V_i(r) = min_e V_{i-1}(r - e) + G_i(e), G_i(e) = the
// device's least cost at w = lb + e (split_full), ties -> the smallest e; the arg-min of every
// (i, r) goes to the wave's LDS strip (kDpLanes bytes per device) for the backtrack. On K1_OK, e
// holds the device's extra layers, as from k1_alloc.
constexpr int kDpLanes = 64;

template <class Rec>
__device__ int k1_dp(const Rec &rec, int M, int R, const Wave &sg, int &e, uint8_t *arg) {
    const int lane = sg.sl;
    double V = kInf;  // lane r: V_{i-1}(r)
    for (int i = 0; i < M; ++i) {
        const auto di = rec.bcast(sg, i).core();
        double G = kInf, g = 0.0;
        int nn = 0, s[4];
        const int wl = rec_wlo(di) + lane;
        if (lane <= R && wl <= rec_whi(di) && split_full(di, wl, g, nn, s)) G = g;
        if (i == 0) {
            V = G;
            continue;
        }
        double best = kInf;
        int be = 0;
        for (int q = 0; q <= R; ++q) {
            const double gq = sg.bcast(G, q);
            const double vp = shfl_f64(V, lane >= q ? lane - q : 0);
            const double c = vp + gq;
            if (lane >= q && c < best) {
                best = c;
                be = q;
            }
        }
        V = lane <= R ? best : kInf;
        arg[i * kDpLanes + lane] = uint8_t(be);
    }
    if (!(sg.bcast(V, R) < kInf)) return K1_INFEASIBLE;
    wave_sync();  // the strip is read across lanes
    int r = R;
    e = 0;
    for (int i = M - 1; i >= 1; --i) {
        const int ei = arg[i * kDpLanes + r];
        if (lane == i) e = ei;
        r -= ei;
    }
    if (lane == 0) e = r;
    return K1_OK;
}

constexpr int kRpSlots = 5;  // row pointers rp[0 .. ncap] per lane: ncap <= 64 * 5 - 1

// Staged decode of one k = 1 instance (M <= 64, lane = device), for a CSR in
// the reference's row order (capacity / link / VRAM rows, then the two cycle
// rows of each device in device order, then the equality row;
// halda_p_solver.py:177-297). Every CSR segment is read with coalesced loads
// into the LDS staging buffer and decoded from there (lane-strided gathers
// straight from HBM touch one cache line per lane and entry):
//   round trip 1  this lane's device columns (c, bounds, integrality) and the
//                 capacity rows' pointers and bounds;
//   round trip 2  the capacity segment's entries, the cycle rows' pointers and bounds;
//   round trip 3  the cycle segment's entries (two halves of <= 64 rows).
// Capacity rows go through decode_cap_row (LDS records, as the generic path);
// the cycle rows of device i are decoded by lanes 2i, 2i + 1 (mod 64) against
// device i's objective entries (shuffled from lane i) and land in lane i's
// registers. Fills d. Returns 0 ok, 1 not a HALDA MILP, 2 not in this shape
// (the caller then runs the generic decode).
__device__ int decode_k1(const halda_batch &B, const WaveCtx &w, unsigned char *scol_raw, unsigned char *sval_raw,
                         const Inst &I, int lane, Dev &d, int &sumlo) {
    const int M = I.M, ncyc = 2 * M, ncap = I.m - 1 - ncyc;
    // M >= 4: the staged 16-B chunks past a segment's end stay inside the equality row
    if (M < 4 || ncap < 0 || ncap > 64 * kCapSlots || ncyc > 64 * kCycSlots) return 2;
    const bool act = lane < M;
    const int64_t co = I.co;
    // ---- round trip 1 (branch-free: out-of-range lanes read a valid element and
    // discard it, so the compiler issues every load before the first wait)
    const int li = act ? lane : 0;
    double cv[6], lbv[6], ubv[6];
    uint8_t ig[6];
#pragma unroll
    for (int b = 0; b < 6; ++b) {
        cv[b] = B.c[co + b * M + li];
        lbv[b] = B.col_lb[co + b * M + li];
        ubv[b] = B.col_ub[co + b * M + li];
        ig[b] = B.integrality[co + b * M + li];
    }
    const double cz = B.c[co + 6 * M + li], lz = B.col_lb[co + 6 * M + li], uz = B.col_ub[co + 6 * M + li];
    const uint8_t iz = B.integrality[co + 6 * M + li];
    const uint8_t iC = B.integrality[co + I.iC];
    const double lC = B.col_lb[co + I.iC], uC = B.col_ub[co + I.iC];
    int rpv[kRpSlots];
    double rub[kCapSlots], rlb[kCapSlots];
#pragma unroll
    for (int j = 0; j < kRpSlots; ++j) rpv[j] = I.rp[min(lane + 64 * j, ncap)];
#pragma unroll
    for (int j = 0; j < kCapSlots; ++j) {
        const int r = min(lane + 64 * j, I.m - 1);
        rub[j] = B.row_ub[I.ro + r];
        rlb[j] = B.row_lb[I.ro + r];
    }
    const int cbase = I.rp[0], cend = I.rp[ncap];
    int dbad = iz != 0 || cz != 0.0 || lz != 0.0 || uz != kInf || lbv[1] < 0.0;
#pragma unroll
    for (int b = 0; b < 6; ++b) dbad |= ig[b] != 1;
#pragma unroll
    for (int j = 0; j < 4; ++j) dbad |= !(cv[2 + j] >= 0.0);
    int bad = act ? dbad : 0;
    const int lo = act ? int(ceil(lbv[0])) : 0;
    if (act) w.cnt[lane] = 0;
    bad |= !(I.kc >= 0.0) || iC != 0 || lC != 0.0 || uC != kInf;
    sumlo = wave_sum(lo);
    HALDA_DSTAMP(1);
    d.cw = cv[0]; d.cn = cv[1]; d.cs0 = cv[2]; d.cs1 = cv[3]; d.cs2 = cv[4]; d.cs3 = cv[5];
    d.wlo = int(ceil(lbv[0]));
    d.whi = int(floor(fmin(ubv[0], I.Wd)));
    d.nlo = int(ceil(lbv[1]));
    d.nhi = int(floor(fmin(ubv[1], I.Wd)));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        d.slo[j] = int(ceil(lbv[2 + j]));
        d.shi[j] = int(floor(fmin(ubv[2 + j], 1e6)));
        d.us[j] = d.vs[j] = 0;
        d.Ks[j] = kNoRow;
    }
    d.uf[0] = d.vf[0] = d.uf[1] = d.vf[1] = 0;
    d.Kf[0] = d.Kf[1] = 0;
    d.r1w = d.r2w = d.rhs1 = d.rhs2 = 0.0;

    // ---- round trip 2: capacity entries (LDS-DMA, coalesced), cycle row pointers / bounds
    const int nc = cend - cbase;
    if (nc < 0 || nc > kStage) return 2;
    const int *scol = reinterpret_cast<const int *>(scol_raw) + stage_lds(B.col_idx + cbase, 4 * nc, scol_raw, lane) / 4;
    const double *sval =
        reinterpret_cast<const double *>(sval_raw) + stage_lds(B.val + cbase, 8 * nc, sval_raw, lane) / 8;
    int yrs[kCycSlots], yre[kCycSlots];
    double yub[kCycSlots], ylb[kCycSlots];
#pragma unroll
    for (int h = 0; h < kCycSlots; ++h) {
        const int r = min(ncap + 64 * h + lane, ncap + ncyc - 1);
        yrs[h] = I.rp[r];
        yre[h] = I.rp[r + 1];
        yub[h] = B.row_ub[I.ro + r];
        ylb[h] = B.row_lb[I.ro + r];
    }
    int hb[kCycSlots], he[kCycSlots];
#pragma unroll
    for (int h = 0; h < kCycSlots; ++h) {
        hb[h] = I.rp[min(ncap + 64 * h, ncap + ncyc)];
        he[h] = I.rp[min(ncap + 64 * h + 64, ncap + ncyc)];
    }
    // row ends of the capacity rows: rp[r + 1] from the next lane (slot j + 1 for lane 63)
    int rpe[kCapSlots];
#pragma unroll
    for (int j = 0; j < kCapSlots; ++j) {
        const int nx = __shfl(rpv[j], (lane + 1) & 63), wrap = __shfl(rpv[j + 1], 0);
        rpe[j] = lane == 63 ? wrap : nx;
    }
    stage_wait();  // staged entries and zeroed counters visible
    HALDA_DSTAMP(2);
#pragma unroll
    for (int j = 0; j < kCapSlots; ++j) {
        const int r = lane + 64 * j;
        if (r < ncap) {
            const int rs = rpv[j] - cbase, nz = rpe[j] - rpv[j];
            if (nz < 1 || rs < 0 || rs + nz > nc) {
                bad |= 1;
            } else if (scol[rs + nz - 1] == I.iC) {
                bad |= 2;  // a cycle row among the capacity rows: another row order
            } else if (rlb[j] != -kInf || nz > kCapNnz || !(fabs(rub[j]) < 1e300)) {
                bad |= 1;
            } else {
                int cols[kCapNnz];
                double vals[kCapNnz];
#pragma unroll
                for (int k = 0; k < kCapNnz; ++k) {
                    cols[k] = k < nz ? scol[rs + k] : -1;
                    vals[k] = k < nz ? sval[rs + k] : 0.0;
                }
                bad |= decode_cap_row<kCapNnz>(w, I, nz, rub[j], cols, vals);
            }
        }
    }

    HALDA_DSTAMP(3);
    // ---- round trip 3 (and 4): cycle segment, two halves of <= 64 rows (32 devices each)
#pragma unroll
    for (int h = 0; h < kCycSlots; ++h) {
        const int rows = min(64, ncyc - 64 * h);
        if (rows <= 0) break;
        const int hn = he[h] - hb[h];
        if (hn < 0 || hn > kStage) return 2;
        wave_sync();  // the previous segment's readers are done
        scol = reinterpret_cast<const int *>(scol_raw) + stage_lds(B.col_idx + hb[h], 4 * hn, scol_raw, lane) / 4;
        sval = reinterpret_cast<const double *>(sval_raw) + stage_lds(B.val + hb[h], 8 * hn, sval_raw, lane) / 8;
        stage_wait();
        if (h == 0) HALDA_DSTAMP(4);
        else HALDA_DSTAMP(5);
        // lane l: row ncap + 64 h + l = cycle row (l & 1) of device 32 h + l / 2
        const int want = 32 * h + (lane >> 1);
        int dev = 0, rb = 0, shape = 0;
        double coef0 = 0.0;
        const bool mine = lane < rows;
        const int rs = yrs[h] - hb[h], nz = yre[h] - yrs[h];
        if (mine) {
            if (nz < 2 || rs < 0 || rs + nz > hn) {
                rb = 1;
            } else {
                const int last = scol[rs + nz - 1];
                const double vlast = sval[rs + nz - 1];
                const int zc = scol[rs + nz - 2];
                const double vz = sval[rs + nz - 2];
                dev = zc - 6 * M;
                if (last != I.iC) shape = 1;  // a capacity row among the cycle rows
                else if (ylb[h] != -kInf || nz > kMaxRowNnz || !(fabs(yub[h]) < 1e300) || vlast != -1.0 ||
                         dev < 0 || dev >= M || fabs(vz) != 1.0)
                    rb = 1;
                else if (dev != want || (vz > 0.0) != ((lane & 1) == 0))
                    shape = 1;  // valid cycle row, another order
            }
        }
        // the device's objective entries (blocks 1..5) from lane dev
        const bool ok = mine && !rb && !shape;
        const int src = ok ? dev : 0;
        double cst[6];
        cst[0] = 0.0;
        cst[1] = shfl_f64(d.cn, src);
        cst[2] = shfl_f64(d.cs0, src);
        cst[3] = shfl_f64(d.cs1, src);
        cst[4] = shfl_f64(d.cs2, src);
        cst[5] = shfl_f64(d.cs3, src);
        if (ok) {
            int seen = 0;
            for (int k = 0; k < nz - 2; ++k) {
                const int j = scol[rs + k];
                const double v = sval[rs + k];
                const int blk = block_of(j, M, I.invM);
                if (j >= 6 * M || j - blk * M != dev) rb = 1;
                else if (blk == 0) coef0 = v;
                else {
                    double cb = cst[1];
#pragma unroll
                    for (int b = 2; b < 6; ++b)
                        if (blk == b) cb = cst[b];
                    rb |= v != cb || ((seen >> blk) & 1);
                    seen |= 1 << blk;
                }
            }
#pragma unroll
            for (int b = 1; b < 6; ++b) rb |= !((seen >> b) & 1) && cst[b] != 0.0;
        }
        bad |= rb | (shape << 1);
        // device i (lanes 32 h .. 32 h + 31) takes rows 2 (i - 32 h) and 2 (i - 32 h) + 1
        const int s0 = (2 * (lane - 32 * h)) & 63, s1 = (s0 + 1) & 63;
        const double c0 = shfl_f64(coef0, s0), c1 = shfl_f64(coef0, s1);
        const double h0 = shfl_f64(yub[h], s0), h1 = shfl_f64(yub[h], s1);
        if (act && lane >= 32 * h && lane < 32 * h + 32) {
            d.r1w = c0;
            d.rhs1 = h0;
            d.r2w = c1;
            d.rhs2 = h1;
        }
    }
    bad = wave_or(bad);
    if (bad) return (bad & 2) ? 2 : 1;
    wave_sync();  // capacity records complete
    // capacity records -> this lane's device (load_dev / check_rows semantics)
    if (act) {
        const int nrow = w.cnt[lane] & 0xff;
        if (nrow > kRows) {
            bad = 1;
        } else {
            int nf = 0;
            for (int q = 0; q < nrow; ++q) {
                const int2 r = w.rows[lane * kRows + q];
                const int kind = (r.x & 0xff) - 1, u = ((r.x >> 8) & 0xff) - 1, v = ((r.x >> 16) & 0xff) - 1;
                if (kind < 0) {
                    if (nf == 0) { d.uf[0] = u; d.vf[0] = v; d.Kf[0] = r.y; }
                    else { d.uf[1] = u; d.vf[1] = v; d.Kf[1] = r.y; }
                    ++nf;
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (kind == j) {
                        bad |= d.Ks[j] != kNoRow && (d.us[j] != u || d.vs[j] != v);  // one (u, v) per slack
                        d.us[j] = u;
                        d.vs[j] = v;
                        d.Ks[j] = max(d.Ks[j], r.y);
                    }
                }
            }
            bad |= nf > 2;
        }
    }
    return wave_or(bad);
}

// One k = 1 instance (lane = device) from decode to x; hands the instance to the
// general kernel (cls = CLS_GEN) when the fast path does not apply.
__device__ void solve_k1(const halda_batch &B, const halda_result &Rz, uint8_t *cls, const WaveCtx &w,
                         unsigned char *scol, unsigned char *sval, const Inst &I, int lane, int *hb_flag,
                         int launch_id) {
    HALDA_STAMP(0);
    Dev d = {};
    int sumlo = 0;
    const int fast = decode_k1(B, w, scol, sval, I, lane, d, sumlo);
    HALDA_PSTAMP(1);
    if (fast == 2) {  // another row order / shape: the general kernel (generic decode) takes it
        if (lane == 0) {
            cls[I.inst] = CLS_GEN1;
            *hb_flag = launch_id;  // the k = 1 general launch of this batch has work
        }
        wave_sync();
        return;
    }
    if (fast == 1) {
        if (lane == 0) write_done(Rz, I.inst, HALDA_STATUS_UNSUPPORTED, 0);
        wave_sync();
        return;
    }
    HALDA_PSTAMP(2);
    HALDA_PSTAMP(3);
    HALDA_PSTAMP(4);
    int e = 0, rounds = 0, nE = 0;
    double gE = 0.0;
    const int rc = k1_alloc(FullRec{d}, I.M, I.W - sumlo, Wave(lane), e, rounds, gE, nE);
    wave_sync();  // LDS records are rewritten by the next instance
    HALDA_PSTAMP(5);
    if (rc == K1_FALLBACK) {
        if (lane == 0) {
            cls[I.inst] = CLS_GEN1;  // the k = 1 general launch (next) takes it
            *hb_flag = launch_id;
        }
        return;
    }
    if (rc == K1_INFEASIBLE) {
        if (lane == 0) write_done(Rz, I.inst, HALDA_STATUS_INFEASIBLE, 1);
        return;
    }
    double g = 0.0, H = 0.0;
    if (lane < I.M) {
        const int wl = d.wlo + e;
        double P, Q;
        int n = 0, s[4] = {0, 0, 0, 0};
        split_full(d, wl, g, n, s);
        dev_cycle(d, wl, n, s, P, Q);
        double *x = Rz.x + I.co;
        const int M = I.M;
        x[lane] = double(wl);
        x[M + lane] = double(n);
        x[2 * M + lane] = double(s[0]);
        x[3 * M + lane] = double(s[1]);
        x[4 * M + lane] = double(s[2]);
        x[5 * M + lane] = double(s[3]);
        x[6 * M + lane] = Q > P ? 0.5 * (Q - P) : 0.0;
        H = Q >= P ? 0.5 * (P + Q) : P;
    }
    const double hmax = fmax(0.0, wave_max(lane < I.M ? H : 0.0));
    const double gsum = wave_sum_f64(lane < I.M ? g : 0.0);
    if (lane == 0) {
        const double obj = gsum + I.kc * hmax;
        Rz.x[I.co + I.iC] = hmax;
        Rz.status[I.inst] = HALDA_STATUS_OPTIMAL;
        Rz.obj_lin[I.inst] = obj;
        Rz.dual_bound[I.inst] = obj;
        Rz.gap[I.inst] = 0.0;
        Rz.nodes[I.inst] = rounds;
    }
    HALDA_STAMP(6);
}

// Screen: four waves per workgroup, each screening kScreenPer consecutive instances.
__global__ __launch_bounds__(256) void halda_screen_kernel(halda_batch B, halda_result Rz, uint8_t *cls, int mmax,
                                                           int r1max, int tab, int tab_kc) {
    const int lane = threadIdx.x & 63;
    const int64_t i0 = (int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6)) * kScreenPer;
    if (i0 >= B.n_inst) return;
    ScreenOut so;
    screen_group(B, Rz, cls, i0, lane, mmax, r1max, tab, tab_kc, so);
}

// k = 1 fast path: persistent 64-thread workgroups (one wave each) over the
// instances the screen classed CLS_K1; wave b owns instances b + j * gridDim.x.
__global__ __launch_bounds__(64, HALDA_K1_WAVES_PER_SIMD) void halda_solve_k1_kernel(halda_batch B, halda_result Rz,
                                                                                      uint8_t *cls, int mmax,
                                                                                      int *hb_flag, int launch_id) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x;
    const K1Slice sl = make_k1_slice(min(mmax, kK1MaxM));
    WaveCtx w = {};
    w.rows = reinterpret_cast<int2 *>(smem + sl.rows);
    w.cyc = reinterpret_cast<double *>(smem + sl.cyc);
    w.cost = reinterpret_cast<double *>(smem + sl.cost);
    w.cnt = reinterpret_cast<int *>(smem + sl.cnt);
    unsigned char *scol = smem + sl.stage;
    unsigned char *sval = smem + sl.stage + kStageColBytes;
    const int S = gridDim.x;
    for (int64_t base = blockIdx.x; base < B.n_inst; base += int64_t(64) * S) {
        const int64_t mine = base + int64_t(lane) * S;
        uint64_t todo = __ballot(mine < B.n_inst && cls[mine] == CLS_K1);
        while (todo) {
            const int bit = __builtin_ctzll(todo);
            todo &= todo - 1;
            Inst I;
            I.inst = int(base + int64_t(bit) * S);
            const int N = B.n_cols[I.inst];
            I.m = B.n_rows[I.inst];
            I.M = (N - 1) / 7;
            I.iC = 7 * I.M;
            I.invM = 1.0f / float(I.M);
            I.co = B.col_off[I.inst];
            I.ro = B.row_off[I.inst];
            I.rp = B.row_ptr + B.csr_off[I.inst];
            I.Wd = B.row_ub[I.ro + I.m - 1];
            I.W = int(I.Wd);
            I.kc = B.c[I.co + I.iC];
            solve_k1(B, Rz, cls, w, scol, sval, I, lane, hb_flag, launch_id);
        }
    }
}

// Screen of ONE instance by one wave (lane = device): the same verdicts as
// screen_group (neither reads the w upper bounds: a device whose w range is
// empty makes the solve report the instance infeasible). Returns the class; settles (and writes) everything but CLS_K1 /
// CLS_GEN. Uniform header values are returned for the solve.
struct Head {
    int N, m, M;
    int64_t co, ro, cs;
    double Wd, kc;
};

__device__ inline int screen_one(const halda_batch &B, const halda_result &Rz, uint8_t *cls, int64_t inst, int lane,
                                 int mmax, int r1max, int tab, int tab_kc, Head &h) {
    h.N = B.n_cols[inst];
    h.m = B.n_rows[inst];
    h.co = B.col_off[inst];
    h.ro = B.row_off[inst];
    h.cs = B.csr_off[inst];
    int status = 0;
    if (h.N < 1 || (h.N - 1) % 7 != 0 || h.m < 1) status = HALDA_STATUS_UNSUPPORTED;
    h.M = status ? 0 : (h.N - 1) / 7;
    if (!status && h.M > mmax) status = HALDA_STATUS_TOO_LARGE;
    const int M = h.M, ma = max(h.m, 1);
    // round trip 2 (branch-free): equality-row extent and bounds, c[C], this lane's w bounds
    const int32_t *rp = B.row_ptr + h.cs;
    const int eqs = rp[ma - 1], eqe = rp[ma];
    const double Wd = B.row_ub[h.ro + ma - 1], Wl = B.row_lb[h.ro + ma - 1];
    const double cC = B.c[h.co + 7 * int64_t(M)];
    const int li = lane < M ? lane : 0;
    const double lb = B.col_lb[h.co + li];  // w upper bounds are left to the solve (decode / tables)
    h.Wd = Wd;
    h.kc = cC;
    if (!status && (!(Wl == Wd) || !(Wd >= 0.0 && Wd < 1e6 && Wd == floor(Wd)) || eqe - eqs != M))
        status = HALDA_STATUS_UNSUPPORTED;
    int verdict = CLS_DONE;
    if (!status) {
        // round trip 3: the equality row (lane = device)
        const int c0 = B.col_idx[eqs + li];
        const double v0 = B.val[eqs + li];
        int bad = 0, infeas = 0, sumlo = 0;
        auto one = [&](int i, int col, double v, double l) {
            bad |= col != i || v != 1.0;
            const int wlo = int(ceil(l));
            infeas |= wlo > int(Wd) || l < 0.0;
            sumlo += wlo;
        };
        if (lane < M) one(lane, c0, v0, lb);
        for (int i = lane + 64; i < M; i += 64) one(i, B.col_idx[eqs + i], B.val[eqs + i], B.col_lb[h.co + i]);
        bad = wave_or(bad | (infeas << 1));
        sumlo = wave_sum(sumlo);
        const int W = int(Wd);
        if (bad & 1) status = HALDA_STATUS_UNSUPPORTED;
        else if ((bad & 2) || sumlo > W || (M == 0 && W > 0)) status = HALDA_STATUS_INFEASIBLE;
        else if (M == 0) status = 1000;  // no devices and W = 0: optimal, x = [C = 0]
        else {
            const int R1 = W - sumlo + 1;
            const bool kc = cC > 0.0;
            if (R1 > r1max || int64_t(M) * odd_stride(R1) > (kc ? tab_kc : tab)) status = HALDA_STATUS_TOO_LARGE;
            else verdict = kc ? CLS_GEN : (M > kK1MaxM ? CLS_GEN1 : CLS_K1);
        }
    }
    if (lane == 0) {
        cls[inst] = uint8_t(verdict);
        if (verdict == CLS_DONE) {
            if (status == 1000) {
                Rz.x[h.co] = 0.0;
                Rz.status[inst] = HALDA_STATUS_OPTIMAL;
                Rz.obj_lin[inst] = Rz.dual_bound[inst] = Rz.gap[inst] = 0.0;
                Rz.nodes[inst] = 0;
            } else {
                write_done(Rz, int(inst), status, 0);
            }
        }
    }
    return verdict;
}

// XCD-aware block -> instance map (bijective for any grid): blocks are dealt round-robin
// over the 8 XCDs (observed placement, speed only), so block b works on instance
// (b % 8) * ~(n / 8) + b / 8 -- each XCD walks one contiguous range of instances in
// order, and the instances of one fleet (adjacent, sharing their CSR) meet in one L2.
__device__ inline int64_t xcd_swizzle(int64_t b, int64_t n) {
    const int64_t x = b % 8, q = n / 8, r = n % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// Screen + k = 1 fast path, one wave per instance: a settled instance's wave
// exits after three round trips, so the hardware dispatcher refills its slot at
// once and the (fewer, longer) solves stay evenly spread over the chip whatever
// the order of the survivors in the batch. k > 1 and wide instances, and the
// fast path's hand-backs, go to halda_solve_kernel (launched next) through cls.
__global__ __launch_bounds__(64, HALDA_K1_WAVES_PER_SIMD) void halda_screen_k1_kernel(halda_batch B, halda_result Rz,
                                                                                       uint8_t *cls, int mmax,
                                                                                       int r1max, int tab, int tab_kc,
                                                                                       int *hb_flag, int launch_id,
                                                                                       int swz) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x;
    const int64_t inst = swz ? xcd_swizzle(blockIdx.x, gridDim.x) : int64_t(blockIdx.x);
    HALDA_WSTAMP(7, __builtin_amdgcn_s_memtime());
    HALDA_WSTAMP(8, __builtin_amdgcn_s_memrealtime());
    Head h;
    if (screen_one(B, Rz, cls, inst, lane, mmax, r1max, tab, tab_kc, h) != CLS_K1) {
        HALDA_WSTAMP(9, __builtin_amdgcn_s_memrealtime());
        return;
    }
    const K1Slice sl = make_k1_slice(min(mmax, kK1MaxM));
    WaveCtx w = {};
    w.rows = reinterpret_cast<int2 *>(smem + sl.rows);
    w.cyc = reinterpret_cast<double *>(smem + sl.cyc);
    w.cost = reinterpret_cast<double *>(smem + sl.cost);
    w.cnt = reinterpret_cast<int *>(smem + sl.cnt);
    Inst I;
    I.inst = int(inst);
    I.m = h.m;
    I.M = h.M;
    I.iC = 7 * h.M;
    I.invM = 1.0f / float(h.M);
    I.co = h.co;
    I.ro = h.ro;
    I.rp = B.row_ptr + h.cs;
    I.Wd = h.Wd;
    I.W = int(h.Wd);
    I.kc = h.kc;
    solve_k1(B, Rz, cls, w, smem + sl.stage, smem + sl.stage + kStageColBytes, I, lane, hb_flag, launch_id);
    HALDA_WSTAMP(9, __builtin_amdgcn_s_memrealtime());
}

// ---------------------------------------------------------------- GPU lowering
// halda_lower_kernel: one wave per fleet, lane = device, writes the fleet's
// fixed-k MILPs for every k-candidate into the halda_batch layout with fixed
// per-fleet strides (solve kernels read them unchanged). Restates the host
// lowering (distilp_amd/solver/lower.py, itself the reference's
// solve_fixed_k_milp, halda_p_solver.py:59-338, with dense_common.py:25-230):
// same row order, same zero-dropping, same FP operation order -> the same CSR
// and vectors bit for bit. An instance with W = L / k < M (every device needs a
// layer: bound-infeasible, 8 of the 9 k at M = 64, L = 80) gets only what the
// screen settles it from: header, w bounds, c[C] and the equality row's bounds.
struct LowerDims {
    int mmax, n_k;
    int64_t cols, rows, nnz;  // strides per instance (cols, rows) and per fleet (nnz)
};

__host__ __device__ inline LowerDims lower_dims(int mmax, int n_k) {
    LowerDims d;
    d.mmax = mmax;
    d.n_k = n_k;
    d.cols = 7 * int64_t(mmax) + 1;
    d.rows = 6 * int64_t(mmax) + 1;   // link M, capacity <= M, VRAM <= 2M, cycle 2M, equality 1
    d.nnz = 26 * int64_t(mmax);       // 2M + 3M + 4M + 16M + M
    return d;
}

// Exclusive prefix sum over the wave (all lanes active); total in *tot.
__device__ inline int wave_excl_scan(int v, int lane, int *tot) {
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    *tot = __shfl(x, 63);
    return x - v;
}

// sum_f_over_s (dense_common.py:49-75) for a key/quantisation known present or absent.
__device__ inline double f_over_s(bool present, double f, double s) {
    return present ? (s > 0.0 ? 0.0 + f / s : 0.0) : 0.0;
}

// Per-device coefficients of the fixed-k MILP (dense_common.py:25-126 and the penalties of
// halda_p_solver.py:195-224) in the reference's operation order; shared by the lowering kernel
// (CSR out) and the sweep kernel (records straight into registers), so both see the same bits.
struct DevCoef {
    double alpha, b, p_bp, p_b, p_v, cst, bcio, xi;
};

// One device's table entry in registers: every field loaded unconditionally (one memory round
// trip for all of them), the coefficients computed from the registers.
struct DevFields {
    double scpu, sgpu, Tc, Tg, tkc, tkg, r2v, v2r, tcomm, sdisk;
    int64_t ram, ccpu, cgpu, cuda, metal, swap;
    int cls, flags;
};

__device__ inline DevFields load_fields(const halda_fleets &F, int64_t g) {
    DevFields f;
    f.scpu = F.scpu_b1[g]; f.sgpu = F.sgpu_b1[g]; f.Tc = F.T_cpu[g]; f.Tg = F.T_gpu[g];
    f.tkc = F.t_kvcpy_cpu[g]; f.tkg = F.t_kvcpy_gpu[g]; f.r2v = F.t_ram2vram[g]; f.v2r = F.t_vram2ram[g];
    f.tcomm = F.t_comm[g]; f.sdisk = F.s_disk[g];
    f.ram = F.d_avail_ram[g]; f.ccpu = F.c_cpu[g]; f.cgpu = F.c_gpu[g]; f.cuda = F.d_avail_cuda[g];
    f.metal = F.d_avail_metal[g]; f.swap = F.swap[g];
    f.cls = F.os_class[g];
    f.flags = F.flags[g];
    return f;
}

__device__ inline DevCoef dev_coef(const halda_model &Mo, const DevFields &F) {
    DevCoef o;
    const double bp = Mo.b_prime;
    const int fl = F.flags;
    const int cls = F.cls;
    const double Tc = F.Tc, tkc = F.tkc, tkg = F.tkg;
    const double cpu = f_over_s(Mo.has_f_q && (fl & HALDA_DEV_CPU_RATE), Mo.f_q_b1, F.scpu);
    const bool hb = fl & HALDA_DEV_GPU;
    const double gpu = hb ? f_over_s(Mo.has_f_q && (fl & HALDA_DEV_GPU_RATE), Mo.f_q_b1, F.sgpu) : 0.0;
    const double tg = hb ? F.Tg : 1.0;
    o.alpha = (cpu + tkc) + (bp / Tc);
    const double beta = hb ? ((gpu - cpu) + (tkg - tkc)) + (bp / tg - bp / Tc) : 0.0;
    o.b = cls == 1 ? 0.0 : beta;
    o.xi = (F.r2v + F.v2r) * ((fl & HALDA_DEV_UMA) ? 0.0 : 1.0);
    const double head = (fl & HALDA_DEV_HEAD) ? 1.0 : 0.0;
    o.bcio = ((Mo.b_in / Mo.V) + Mo.b_out) * head + double(F.ccpu);
    const double sd = fmax(1.0, F.sdisk);
    o.p_bp = bp / sd;
    o.p_b = Mo.b_layer / sd;
    o.p_v = cls == 2 ? o.p_b : o.p_bp;
    o.cst = o.xi + F.tcomm;
    return o;
}

__device__ inline DevCoef dev_coef(const halda_model &Mo, const halda_fleets &F, int64_t g) {
    return dev_coef(Mo, load_fields(F, g));
}

// Right-hand sides of the capacity rows (halda_p_solver.py:227-277).
__device__ inline double rhs_ram(const DevFields &F, int set, double bcio) {
    if (set == 1) return double(F.ram) - bcio;
    if (set == 2) return double(F.metal) - bcio - double(F.cgpu);
    return double(F.ram + F.swap) - bcio;
}
__device__ inline double rhs_cuda(const DevFields &F) { return double(F.cuda) - double(F.cgpu); }
__device__ inline double rhs_metal(const halda_model &Mo, const DevFields &F) {
    const double head = (F.flags & HALDA_DEV_HEAD) ? 1.0 : 0.0;
    return double(F.metal) - double(F.cgpu) - Mo.b_out * head;
}
__device__ inline double rhs_ram(const halda_fleets &F, int64_t g, int set, double bcio) {
    return rhs_ram(load_fields(F, g), set, bcio);
}
__device__ inline double rhs_cuda(const halda_fleets &F, int64_t g) { return rhs_cuda(load_fields(F, g)); }
__device__ inline double rhs_metal(const halda_model &Mo, const halda_fleets &F, int64_t g) {
    return rhs_metal(Mo, load_fields(F, g));
}

// Objective constants of one fleet (lane-parallel loads, the reference's sequential sums over
// readlane): sum t_comm and sum xi in device order, kappa (dense_common.py:211-230) with its
// M1 part before its M3 part (:226). Uniform on every lane.
__device__ inline void fleet_offsets(const halda_model &Mo, const halda_fleets &F, int64_t d0, int M, int lane,
                                     double &tsum, double &xsum, double &kappa) {
    tsum = 0.0;
    xsum = 0.0;
    double tail1 = 0.0;
    int hi = -1;
    for (int i0 = 0; i0 < M; i0 += 64) {
        const int i = min(i0 + lane, M - 1);
        const int64_t g = d0 + i;
        const double tc = F.t_comm[g];
        const double xv = (F.t_ram2vram[g] + F.t_vram2ram[g]) * ((F.flags[g] & HALDA_DEV_UMA) ? 0.0 : 1.0);
        const int cls = F.os_class[g];
        const double tl = double(F.c_cpu[g] - F.d_avail_ram[g] - F.swap[g]) / F.s_disk[g];
        const uint64_t heads = __ballot(i0 + lane < M && (F.flags[g] & HALDA_DEV_HEAD));
        if (hi < 0 && heads) hi = i0 + __builtin_ctzll(heads);
        const int n = min(64, M - i0);
        for (int q = 0; q < n; ++q) {
            tsum += bcast(tc, q);
            xsum += bcast(xv, q);
            const int cq = bcast(cls, q);
            if (cq == 1) tail1 += bcast(tl, q);
        }
    }
    double tail = tail1;
    for (int i0 = 0; i0 < M; i0 += 64) {
        const int i = min(i0 + lane, M - 1);
        const int64_t g = d0 + i;
        const int cls = F.os_class[g];
        const double tl = double(F.c_cpu[g] - F.d_avail_ram[g] - F.swap[g]) / F.s_disk[g];
        const int n = min(64, M - i0);
        for (int q = 0; q < n; ++q)
            if (bcast(cls, q) == 3) tail += bcast(tl, q);
    }
    const int64_t h = d0 + (hi < 0 ? 0 : hi);
    double total = f_over_s(Mo.has_f_out && (F.flags[h] & HALDA_DEV_CPU_RATE), Mo.f_out_b1, F.scpu_b1[h]);
    total += (Mo.b_in / Mo.V + Mo.b_out) / F.T_cpu[h];
    total += Mo.b_in / (Mo.V * F.s_disk[h]);
    total += Mo.b_out / F.s_disk[h];
    kappa = total + tail;
}

struct LowerOut {
    halda_batch b;         // arrays written (device pointers, const-cast by the kernel)
    int32_t *n_cols, *n_rows, *row_ptr, *col_idx;
    int64_t *csr_off, *col_off, *row_off;
    double *val, *c, *col_lb, *col_ub, *row_lb, *row_ub, *offs;  // offs[f]: t_comm sum, xi sum, kappa
    uint8_t *integrality;
};

__global__ __launch_bounds__(64) void halda_lower_kernel(halda_model Mo, halda_fleets F, const int32_t *ks, int n_k,
                                                         LowerDims D, LowerOut O) {
    const int lane = threadIdx.x;
    const int f = blockIdx.x;
    if (f >= F.n_fleets) return;
    const int64_t d0 = F.dev_off[f];
    const int M = int(F.dev_off[f + 1] - d0);
    const int64_t nnz0 = int64_t(f) * D.nnz;       // this fleet's CSR entries
    const int64_t rp0 = int64_t(f) * (D.rows + 1);  // this fleet's row_ptr segment
    const double bp = Mo.b_prime;
    const int iC = 7 * M;
    int rows = 0;
    int64_t nnz = 0;
    // per-block row emission: lane i emits up to 2 rows for device i (chunks of 64). Two passes of the
    // row function: count the nonzeros, scan, then write the entries straight to the CSR (no private
    // arrays: dynamically indexed ones would live in scratch).
    auto emit = [&](auto &&row_fn) {
        for (int i0 = 0; i0 < M; i0 += 64) {
            const int i = i0 + lane;
            const bool act = i < M;
            int c0 = 0, c1 = 0;
            double r0 = 0.0, r1 = 0.0;
            const int nr = act ? row_fn(i, false, c0, c1, r0, r1, int64_t(0), int64_t(0)) : 0;
            int rtot = 0, ntot = 0;
            const int rbase = wave_excl_scan(nr, lane, &rtot);
            const int nbase = wave_excl_scan(c0 + c1, lane, &ntot);
            if (nr > 0) {
                const int64_t e0 = nnz0 + nnz + nbase, e1 = e0 + c0;
                int w0 = 0, w1 = 0;
                row_fn(i, true, w0, w1, r0, r1, e0, e1);
                const int r = rows + rbase;
                O.row_ptr[rp0 + r] = int32_t(e0);
                if (nr > 1) O.row_ptr[rp0 + r + 1] = int32_t(e1);
                for (int j = 0; j < n_k; ++j) {
                    if (Mo.L / ks[j] < M) continue;  // bound-infeasible: the screen reads only the eq row
                    const int64_t ro = (int64_t(f) * n_k + j) * D.rows;
                    O.row_lb[ro + r] = -kInf;
                    O.row_ub[ro + r] = r0;
                    if (nr > 1) {
                        O.row_lb[ro + r + 1] = -kInf;
                        O.row_ub[ro + r + 1] = r1;
                    }
                }
            }
            rows += rtot;
            nnz += ntot;
        }
    };
    // one (col, val) of a row when val != 0 (scipy builds its CSC from the dense rows): counted, or
    // written at e + n when wr
    auto put = [&](bool wr, int64_t e, int &n, int col, double v) {
        if (v != 0.0) {
            if (wr) {
                O.col_idx[e + n] = col;
                O.val[e + n] = v;
            }
            ++n;
        }
    };
    // ---- per-device coefficients (lower._device_arrays order); lane i's own device is computed once
    DevCoef mine = {};
    if (lane < M) mine = dev_coef(Mo, F, d0 + lane);
    auto coeff = [&](int i, double &alpha, double &b, double &p_bp, double &p_b, double &p_v, double &cst,
                     double &bcio, double &xi) {
        const DevCoef c = i == lane ? mine : dev_coef(Mo, F, d0 + i);
        alpha = c.alpha; b = c.b; p_bp = c.p_bp; p_b = c.p_b; p_v = c.p_v; cst = c.cst; bcio = c.bcio; xi = c.xi;
    };
    // 1. link rows n_i - w_i <= 0
    emit([&](int i, bool wr, int &c0, int &c1, double &r0, double &r1, int64_t e0, int64_t e1) {
        (void)c1; (void)r1; (void)e1;
        put(wr, e0, c0, i, -1.0);
        put(wr, e0, c0, M + i, 1.0);
        r0 = 0.0;
        return 1;
    });
    // 2-4. RAM / Metal capacity rows by set
    for (int set = 1; set <= 3; ++set) {
        emit([&](int i, bool wr, int &c0, int &c1, double &r0, double &r1, int64_t e0, int64_t e1) {
            (void)c1; (void)r1; (void)e1;
            const int64_t g = d0 + i;
            if (F.os_class[g] != set) return 0;
            if (set == 2 && !(F.flags[g] & HALDA_DEV_METAL_AVAIL)) return 0;
            double alpha, b, p_bp, p_b, p_v, cst, bcio, xi;
            coeff(i, alpha, b, p_bp, p_b, p_v, cst, bcio, xi);
            put(wr, e0, c0, i, bp);
            if (set == 3) put(wr, e0, c0, M + i, -bp);
            put(wr, e0, c0, (1 + set) * M + i, -bp);
            r0 = rhs_ram(F, g, set, bcio);
            return 1;
        });
    }
    // 5. VRAM rows: per device the CUDA row, then the Metal row
    emit([&](int i, bool wr, int &c0, int &c1, double &r0, double &r1, int64_t e0, int64_t e1) {
        const int64_t g = d0 + i;
        const uint8_t fl = F.flags[g];
        const bool cu = fl & HALDA_DEV_CUDA_OK, me = fl & HALDA_DEV_METAL_OK;
        const double rc = rhs_cuda(F, g);
        const double rm = rhs_metal(Mo, F, g);
        if (cu) {
            put(wr, e0, c0, M + i, bp);
            put(wr, e0, c0, 5 * M + i, -bp);
            r0 = rc;
        }
        if (me) {
            int &cm = cu ? c1 : c0;
            const int64_t em = cu ? e1 : e0;
            put(wr, em, cm, M + i, bp);
            put(wr, em, cm, 5 * M + i, -bp);
            (cu ? r1 : r0) = rm;
        }
        return int(cu) + int(me);
    });
    // 6. cycle rows busy + z - C <= -const ; busy + F - z - C <= -const
    emit([&](int i, bool wr, int &c0, int &c1, double &r0, double &r1, int64_t e0, int64_t e1) {
        double alpha, b, p_bp, p_b, p_v, cst, bcio, xi;
        coeff(i, alpha, b, p_bp, p_b, p_v, cst, bcio, xi);
        put(wr, e0, c0, i, alpha);
        put(wr, e1, c1, i, alpha + p_bp);
        put(wr, e0, c0, M + i, b);
        put(wr, e1, c1, M + i, b);
        put(wr, e0, c0, 2 * M + i, p_bp);
        put(wr, e1, c1, 2 * M + i, p_bp);
        put(wr, e0, c0, 3 * M + i, p_b);
        put(wr, e1, c1, 3 * M + i, p_b);
        put(wr, e0, c0, 4 * M + i, p_bp);
        put(wr, e1, c1, 4 * M + i, p_bp);
        put(wr, e0, c0, 5 * M + i, p_v);
        put(wr, e1, c1, 5 * M + i, p_v);
        put(wr, e0, c0, 6 * M + i, 1.0);
        put(wr, e1, c1, 6 * M + i, -1.0);
        put(wr, e0, c0, iC, -1.0);
        put(wr, e1, c1, iC, -1.0);
        r0 = r1 = -cst;
        return 2;
    });
    // 7. equality row sum_i w_i = W (row bounds per k below)
    {
        const int r = rows;
        O.row_ptr[rp0 + r] = int32_t(nnz0 + nnz);
        for (int i = lane; i < M; i += 64) {
            O.col_idx[nnz0 + nnz + i] = i;
            O.val[nnz0 + nnz + i] = 1.0;
        }
        nnz += M;
        rows += 1;
        if (lane == 0) O.row_ptr[rp0 + rows] = int32_t(nnz0 + nnz);
    }
    // ---- per-instance vectors (lane = device) and headers
    for (int i0 = 0; i0 < M; i0 += 64) {
        const int i = i0 + lane;
        if (i >= M) continue;
        const int64_t g = d0 + i;
        const uint8_t fl = F.flags[g];
        const int cls = F.os_class[g];
        double alpha, b, p_bp, p_b, p_v, cst, bcio, xi;
        coeff(i, alpha, b, p_bp, p_b, p_v, cst, bcio, xi);
        const double busy[6] = {alpha, b, p_bp, p_b, p_bp, p_v};
        const double gpu = (fl & (HALDA_DEV_CUDA_OK | HALDA_DEV_METAL_OK)) ? 1.0 : 0.0;
        const double scale[6] = {1.0, gpu, cls == 1 ? 1.0 : 0.0, cls == 2 ? 1.0 : 0.0, cls == 3 ? 1.0 : 0.0, gpu};
        for (int j = 0; j < n_k; ++j) {
            const double W = double(Mo.L / ks[j]);
            const int64_t co = (int64_t(f) * n_k + j) * D.cols;
            if (Mo.L / ks[j] < M) {
                // W < M = sum lb(w): the screen settles it from the w bounds (and c[C], the eq row)
                O.col_lb[co + i] = 1.0;
                O.col_ub[co + i] = W;
                continue;
            }
#pragma unroll
            for (int blk = 0; blk < 6; ++blk) {
                O.c[co + blk * M + i] = busy[blk];
                O.col_lb[co + blk * M + i] = blk == 0 ? 1.0 : 0.0;
                O.col_ub[co + blk * M + i] = scale[blk] * W;
                O.integrality[co + blk * M + i] = 1;
            }
            O.c[co + 6 * M + i] = 0.0;
            O.col_lb[co + 6 * M + i] = 0.0;
            O.col_ub[co + 6 * M + i] = kInf;
            O.integrality[co + 6 * M + i] = 0;
        }
    }
    for (int j = lane; j < n_k; j += 64) {
        const int64_t inst = int64_t(f) * n_k + j;
        const int64_t co = inst * D.cols, ro = inst * D.rows;
        const double W = double(Mo.L / ks[j]);
        O.c[co + iC] = double(ks[j] - 1);
        O.col_lb[co + iC] = 0.0;
        O.col_ub[co + iC] = kInf;
        O.integrality[co + iC] = 0;
        O.row_lb[ro + rows - 1] = W;
        O.row_ub[ro + rows - 1] = W;
        O.n_cols[inst] = 7 * M + 1;
        O.n_rows[inst] = rows;
        O.csr_off[inst] = rp0;
        O.col_off[inst] = co;
        O.row_off[inst] = ro;
    }
    // ---- objective offsets: sum t_comm and sum xi in device order, kappa (dense_common.py:211-230)
    double tsum, xsum, kappa;
    fleet_offsets(Mo, F, d0, M, lane, tsum, xsum, kappa);
    if (lane == 0) {
        O.offs[3 * f + 0] = tsum;
        O.offs[3 * f + 1] = xsum;
        O.offs[3 * f + 2] = kappa;
    }
}

// ---------------------------------------------------------------- fused k-sweep
// halda_sweep_kernel: the whole `halda_solve` k-sweep of a fleet (halda_p_solver.py:369-436) in
// one wave, from the fleet's device-field table, without materialising the MILPs. For every
// k-candidate the wave builds, per device, exactly the record that decoding the lowered CSR
// yields (load_dev of decode_cap_row / decode_cycle_row output, with the same rejections),
// straight from the coefficients the lowering kernel writes into the CSR (dev_coef / rhs_* are
// shared, so the values are the same bits); then settles bound-infeasible k (L / k < M), solves
// k = 1 by the register greedy of the k = 1 fast path and the rest (k > 1, fleets wider than
// 64 devices, fast-path fallbacks) by the general kernel's tables + DP / threshold scan, and keeps
// the best k by the reference's rule (ascending k, strict "<" on obj_value, :407) in registers.
// obj_value = c.x + sum t_comm + sum xi + kappa is formed in a fixed order (per-device costs
// summed by a wave reduction, + (k - 1) C, + the fleet constants).
//
// kTables = false: no LDS; a fleet that needs a table is flagged (fflag[f] = 1, hb_flag = launch)
// and left to the next launch. kTables = true: tables in the LDS slice (kGlobal = false) or in a
// per-wave global slice (kGlobal = true); want = 1 selects the flagged fleets only (gated on the
// hand-back flag), want = 0 every fleet.

// Device record of table entry g, compact: the five coefficients, the least-slack offsets of its
// RAM / Metal row and of its VRAM rows, its class and GPU flag; W = L / k is set per k. dev()
// expands it to exactly the Dev that decoding the lowered CSR gives (load_dev of decode_cap_row /
// decode_cycle_row output), so the solve code is shared; bad = 1 where decode would reject.
struct FieldRec {
    double alpha, b, p_bp, p_b, cst;
    int Kset, Kvram;  // kNoRow: the row is absent
    int cls, gpu, W;
    __device__ inline Dev dev() const {
        Dev d;
        d.cw = alpha; d.cn = b; d.cs0 = p_bp; d.cs1 = p_b; d.cs2 = p_bp; d.cs3 = cls == 2 ? p_b : p_bp;
        // cycle rows: busy + z - C <= -cst, busy + F - z - C <= -cst (w entries alpha, alpha + b'/s_disk)
        d.r1w = alpha;
        d.r2w = alpha + p_bp;
        d.rhs1 = -cst;
        d.rhs2 = -cst;
        d.wlo = 1; d.whi = W; d.nlo = 0; d.nhi = gpu ? W : 0;
        const bool hs = Kset != kNoRow, hv = Kvram != kNoRow;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const bool mine = cls == j + 1;
            d.slo[j] = 0;
            d.shi[j] = mine ? W : 0;
            d.us[j] = mine && hs ? 1 : 0;
            d.vs[j] = j == 2 && mine && hs ? -1 : 0;
            d.Ks[j] = mine ? Kset : kNoRow;
        }
        d.slo[3] = 0; d.shi[3] = gpu ? W : 0; d.us[3] = 0; d.vs[3] = hv ? 1 : 0; d.Ks[3] = Kvram;
        // the link row n - w <= 0 (scale 1: K = floor(0 + 1e-9) = 0)
        d.uf[0] = -1; d.vf[0] = 1; d.Kf[0] = 0;
        d.uf[1] = 0; d.vf[1] = 0; d.Kf[1] = 0;
        return d;
    }
    __device__ inline FieldRec shfl(int src) const {  // per-lane source (all lanes active)
        FieldRec o;
        o.alpha = shfl_f64(alpha, src); o.b = shfl_f64(b, src); o.p_bp = shfl_f64(p_bp, src);
        o.p_b = shfl_f64(p_b, src); o.cst = shfl_f64(cst, src);
        o.Kset = __shfl(Kset, src); o.Kvram = __shfl(Kvram, src);
        const int cg = __shfl(cls | (gpu << 4), src);
        o.cls = cg & 15; o.gpu = cg >> 4;
        o.W = W;
        return o;
    }
    template <class SG>
    __device__ inline auto bcast(const SG &sg, int src) const;  // the problem's device src, on every lane
    __device__ inline const FieldRec &core() const { return *this; }
};

// A record broadcast to the whole problem (every lane holds device src's record): its split takes
// the branches on the record's shape instead of selects (they are uniform here), skipping the
// candidates the device does not have; the same candidates, order and tie rule as on a FieldRec.
struct UFieldRec : FieldRec {
    __device__ inline const UFieldRec &core() const { return *this; }
};

template <class SG>
__device__ inline auto FieldRec::bcast(const SG &sg, int src) const {
    UFieldRec o;
    o.alpha = sg.bcast(alpha, src); o.b = sg.bcast(b, src); o.p_bp = sg.bcast(p_bp, src);
    o.p_b = sg.bcast(p_b, src); o.cst = sg.bcast(cst, src);
    o.Kset = sg.bcast(Kset, src); o.Kvram = sg.bcast(Kvram, src);
    const int cg = sg.bcast(cls | (gpu << 4), src);
    o.cls = cg & 15; o.gpu = cg >> 4;
    o.W = W;
    return o;
}

// The solve primitives on a FieldRec, specialised. The Dev that dev() expands a record to has two
// live slacks: its class slack s_c >= w + Kset (class 3: w - n + Kset; s_c <= W) and the VRAM slack
// t >= n + Kvram (t <= nhi), both priced pv = (class 2 ? p_b : p_bp), with 0 <= n <= min(w, nhi),
// nhi = W on a GPU device, else 0; every other slack is pinned to 0 by its bounds. So split_full /
// split_step / dev_cycle below visit the same candidates with the same tie rule as on dev() and give
// the same bits: a pinned slack adds p * 0 = +0, which leaves any sum of terms >= +0 unchanged, and
// where that term is NaN there (an infinite price of another class: inf * 0) the cost is NaN here.
__device__ inline double rec_pv(const FieldRec &r) { return r.cls == 2 ? r.p_b : r.p_bp; }
__device__ inline bool rec_own(const FieldRec &r) { return unsigned(r.cls - 1) < 3u; }
__device__ inline bool rec_nanx(const FieldRec &r) { return r.p_bp == kInf || (r.p_b == kInf && r.cls != 2); }
__device__ inline int rec_wlo(const FieldRec &) { return 1; }
__device__ inline int rec_whi(const FieldRec &r) { return r.W; }

// Feasible n-interval for w layers (n_interval on dev()); false when no n is feasible (also when
// the class 1 / 2 slack, which does not depend on n, exceeds its bound).
__device__ inline bool rec_interval(const FieldRec &r, int w, int &nL, int &nU) {
    const bool hs = r.Kset != kNoRow;
    const int nhi = r.gpu ? r.W : 0;
    nL = r.cls == 3 && hs ? max(0, w + r.Kset - r.W) : 0;
    nU = min(nhi, w);
    nU = r.Kvram != kNoRow ? min(nU, nhi - r.Kvram) : nU;
    const bool setok = !(hs && (r.cls == 1 || r.cls == 2)) || max(0, w + r.Kset) <= r.W;
    return nL <= nU && setok;
}

// One candidate n of a split, branch-free (selects, non-short-circuit tests): dev_cost on dev() for
// (w, n) and its least slacks (sc = the class slack, t = VRAM), in dev_cost's term order (aw = alpha
// w, pv = rec_pv, own = rec_own), and the tie rule "smaller cost, then smaller n". The record's NaN
// flag (rec_nanx) is applied by the caller: it fails the whole split, as a NaN cost at every
// candidate does.
__device__ inline void rec_try(const FieldRec &r, double aw, double pv, bool own, int w, int nn, int nL, int nU,
                               double &best, int &bn) {
    nn = min(max(nn, nL), nU);
    const int sc = max(0, w - (r.cls == 3 ? nn : 0) + r.Kset), t = max(0, nn + r.Kvram);  // kNoRow: 0
    double g = aw;
    g = g + r.b * double(nn);
    const double gs = g + pv * double(sc);
    g = own ? gs : g;
    g = g + pv * double(t);
    const bool better = (g < best) | ((g == best) & (nn < bn));
    best = better ? g : best;
    bn = better ? nn : bn;
}

__device__ inline void rec_slacks(const FieldRec &r, int w, int n, int s[4]) {
    const int sc = max(0, w - (r.cls == 3 ? n : 0) + r.Kset);
    s[0] = r.cls == 1 ? sc : 0;
    s[1] = r.cls == 2 ? sc : 0;
    s[2] = r.cls == 3 ? sc : 0;
    s[3] = max(0, n + r.Kvram);
}

// split_full on dev(): candidates nL, nU, the class-slack kink (class 3) and the VRAM kink, in that
// order. Every candidate is evaluated on every lane (no divergent branches); an absent kink re-tries
// nL, which never changes (best, bn): after nL's own try either bn = nL or best < cost(nL), and no
// candidate lies below nL.
template <bool kUniform>
__device__ inline bool split_full_impl(const FieldRec &r, int w, double &g, int &n, int s[4]) {
    int nL, nU;
    const bool okI = rec_interval(r, w, nL, nU);
    const double pv = rec_pv(r), aw = r.alpha * double(w);
    const bool own = rec_own(r);
    double best = kInf;
    int bn = -1;
    rec_try(r, aw, pv, own, w, nL, nL, nU, best, bn);
    rec_try(r, aw, pv, own, w, nU, nL, nU, best, bn);
    const bool hc = r.cls == 3 && r.Kset != kNoRow, hv = r.Kvram != kNoRow;
    if (!kUniform || hc) rec_try(r, aw, pv, own, w, hc ? w + r.Kset : nL, nL, nU, best, bn);  // class-slack kink
    if (!kUniform || hv) rec_try(r, aw, pv, own, w, hv ? -r.Kvram : nL, nL, nU, best, bn);     // VRAM kink
    const bool ok = okI & (bn >= 0) & !rec_nanx(r);
    if (ok) {
        g = best;
        n = bn;
        rec_slacks(r, w, bn, s);
    }
    return ok;
}
__device__ inline bool split_full(const FieldRec &r, int w, double &g, int &n, int s[4]) {
    return split_full_impl<false>(r, w, g, n, s);
}
// split_full at w = 1 (the record's lower bound): 0 <= nL <= n <= nU <= w = 1, so every kink clamps
// to nL or nU and re-trying either is a no-op (after nU's try best <= cost(nU), and on a tie bn <= nU):
// the two end tries give split_full's result.
__device__ inline bool split_first(const FieldRec &r, int w, double &g, int &n, int s[4]) {
    if (w != 1) return split_full(r, w, g, n, s);
    int nL, nU;
    const bool okI = rec_interval(r, w, nL, nU);
    const double pv = rec_pv(r), aw = r.alpha * double(w);
    const bool own = rec_own(r);
    double best = kInf;
    int bn = -1;
    rec_try(r, aw, pv, own, w, nL, nL, nU, best, bn);
    rec_try(r, aw, pv, own, w, nU, nL, nU, best, bn);
    const bool ok = okI & (bn >= 0) & !rec_nanx(r);
    if (ok) {
        g = best;
        n = bn;
        rec_slacks(r, w, bn, s);
    }
    return ok;
}
__device__ inline bool split_full(const UFieldRec &r, int w, double &g, int &n, int s[4]) {
    return split_full_impl<true>(r, w, g, n, s);
}

__device__ inline bool split_step(const FieldRec &r, int w, int n_prev, double &g, int &n, int s[4]) {
    int nL, nU;
    const bool okI = rec_interval(r, w, nL, nU);
    const double pv = rec_pv(r), aw = r.alpha * double(w);
    const bool own = rec_own(r);
    double best = kInf;
    int bn = -1;
    rec_try(r, aw, pv, own, w, n_prev, nL, nU, best, bn);
    rec_try(r, aw, pv, own, w, n_prev + 1, nL, nU, best, bn);
    const bool ok = okI & (bn >= 0) & !rec_nanx(r);
    if (ok) {
        g = best;
        n = bn;
        rec_slacks(r, w, bn, s);
    }
    return ok;
}

// dev_cycle on dev(): rows (alpha, alpha + p_bp) w + b n + slack terms <= -cst.
__device__ inline void dev_cycle(const FieldRec &r, int w, int n, const int s[4], double &P, double &Q) {
    const double pv = rec_pv(r);
    const int sc = r.cls == 1 ? s[0] : r.cls == 2 ? s[1] : s[2];
    const double t0 = r.b * double(n), tc = pv * double(sc), tv = pv * double(s[3]);
    double a1 = r.alpha * double(w), a2 = (r.alpha + r.p_bp) * double(w);
    a1 = a1 + t0; a2 = a2 + t0;
    const bool own = rec_own(r);
    const double o1 = a1 + tc, o2 = a2 + tc;
    a1 = own ? o1 : a1;
    a2 = own ? o2 : a2;
    a1 = a1 + tv; a2 = a2 + tv;
    const bool nanx = rec_nanx(r);
    a1 = nanx ? __builtin_nan("") : a1;
    a2 = nanx ? __builtin_nan("") : a2;
    P = a1 - (-r.cst);
    Q = a2 - (-r.cst);
}

__device__ inline double least_cycle(const FieldRec &r, int w, int n, const int s[4]) {
    double P, Q;
    dev_cycle(r, w, n, s, P, Q);
    return Q >= P ? 0.5 * (P + Q) : P;
}

__device__ inline FieldRec field_rec(const halda_model &Mo, const DevFields &F, int &bad) {
    FieldRec r;
    const DevCoef c = dev_coef(Mo, F);
    const double bp = Mo.b_prime;
    const int fl = F.flags;
    r.alpha = c.alpha; r.b = c.b; r.p_bp = c.p_bp; r.p_b = c.p_b; r.cst = c.cst;
    r.cls = F.cls;
    r.gpu = (fl & (HALDA_DEV_CUDA_OK | HALDA_DEV_METAL_OK)) ? 1 : 0;
    r.W = 0;
    r.Kset = r.Kvram = kNoRow;
    bad = !(fabs(c.cst) < 1e300);  // cycle-row rhs
    bad |= !(c.p_bp >= 0.0) || !(c.p_b >= 0.0) || !(r.cls == 2 ? c.p_b >= 0.0 : c.p_bp >= 0.0);  // slack prices
    // capacity rows b' u w + b' v n - b' s <= rhs -> s >= u w + v n + ceil(-rhs / b' - eps)
    auto K = [&](double rhs, int &dst) {
        if (!(bp > 0.0) || !(fabs(rhs) < 1e300)) {
            bad = 1;
            return;
        }
        const double kk = ceil(-rhs / bp - kSlackEps);
        if (!(fabs(kk) < 1e8)) {
            bad = 1;
            return;
        }
        dst = max(dst, int(kk));
    };
    if (r.cls == 1 || r.cls == 3 || (fl & HALDA_DEV_METAL_AVAIL)) K(rhs_ram(F, r.cls, c.bcio), r.Kset);
    // VRAM rows: CUDA or Metal (one division for either; both rows only on a device with both)
    const bool cu = fl & HALDA_DEV_CUDA_OK, mt = fl & HALDA_DEV_METAL_OK;
    if (cu && mt) {
        K(rhs_cuda(F), r.Kvram);
        K(rhs_metal(Mo, F), r.Kvram);
    } else if (cu || mt) {
        K(cu ? rhs_cuda(F) : rhs_metal(Mo, F), r.Kvram);
    }
    return r;
}

// Device records of a fleet straight from its table (the sweep's table path).
// Device records of a fleet for the sweep's table path: for M <= 64 lane i already holds device
// i's record (me), which other lanes fetch by shuffle; wider fleets rebuild it from the table.
// load() runs on every lane (uniform control flow: the shuffles read every lane's registers).
struct FieldSrc {
    using Rec = FieldRec;
    const halda_model *Mo;
    const halda_fleets *F;
    const FieldRec *me;  // lane's own record (M <= lanes per problem), or nullptr
    int64_t d0;
    int W;
    int base;            // first lane of the problem's lane group
    __device__ inline void load(FieldRec &r, const WaveCtx &, int i) const {
        if (me) {
            r = me->shfl(base + i);
        } else {
            int bad = 0;
            r = field_rec(*Mo, load_fields(*F, d0 + i), bad);
        }
        r.W = W;
    }
};

// Objective constants of a fleet for the sweep's own obj_value (a fixed tree order: wave
// reductions): sum t_comm, sum xi, kappa with the head's terms (dense_common.py:211-230). For
// M <= 64 lane i passes device i's fields (in registers) and the head's come by readlane.
__device__ inline double tail_term(const DevFields &f) {
    return f.cls != 2 ? double(f.ccpu - f.ram - f.swap) / f.sdisk : 0.0;
}
__device__ inline double xi_term(const DevFields &f) { return (f.r2v + f.v2r) * ((f.flags & HALDA_DEV_UMA) ? 0.0 : 1.0); }

__device__ inline double kappa_head(const halda_model &Mo, int flags, double scpu, double Tc, double sdisk) {
    double total = f_over_s(Mo.has_f_out && (flags & HALDA_DEV_CPU_RATE), Mo.f_out_b1, scpu);
    total += (Mo.b_in / Mo.V + Mo.b_out) / Tc;
    total += Mo.b_in / (Mo.V * sdisk);
    total += Mo.b_out / sdisk;
    return total;
}

template <class SG>
__device__ inline void fleet_offsets_regs(const halda_model &Mo, const DevFields &mf, int M, const SG &sg, double &tsum,
                                          double &xsum, double &kappa) {
    const bool act = sg.sl < M;
    // one wave sum for the three per-device constants of obj_value (t_comm, xi and kappa's tail term,
    // added per device in that order): tsum carries all of it, xsum is 0 and kappa its head terms;
    // obj_value's constants are summed in this fixed order (the host recomputes the reference's own
    // order for halda_solve)
    tsum = sg.sum_f64(act ? (mf.tcomm + xi_term(mf)) + tail_term(mf) : 0.0);
    xsum = 0.0;
    int hi = sg.lowest(act && (mf.flags & HALDA_DEV_HEAD));
    if (hi >= SG::S) hi = 0;
    // kappa_head's four quotients on lanes 0..3 of the problem (one division for the four), summed in
    // its order
    const int hf = sg.bcast(mf.flags, hi);
    const double scpu = sg.bcast(mf.scpu, hi), Tc = sg.bcast(mf.Tc, hi), sdisk = sg.bcast(mf.sdisk, hi);
    const double bv = Mo.b_in / Mo.V;
    const int j = sg.sl & 3;
    const double num = j == 0 ? Mo.f_out_b1 : j == 1 ? bv + Mo.b_out : j == 2 ? Mo.b_in : Mo.b_out;
    const double den = j == 0 ? scpu : j == 1 ? Tc : j == 2 ? Mo.V * sdisk : sdisk;
    const double q = num / den;
    const double q0 = sg.bcast(q, 0), q1 = sg.bcast(q, 1), q2 = sg.bcast(q, 2), q3 = sg.bcast(q, 3);
    double total = (Mo.has_f_out && (hf & HALDA_DEV_CPU_RATE)) ? (scpu > 0.0 ? 0.0 + q0 : 0.0) : 0.0;
    total += q1;
    total += q2;
    total += q3;
    kappa = total;
}

__device__ inline void fleet_offsets_tree(const halda_model &Mo, const halda_fleets &F, int64_t d0, int M, int lane,
                                          double &tsum, double &xsum, double &kappa) {
    double t = 0.0, x = 0.0, tail = 0.0;
    int hi = 0x7fffffff;
    for (int i = lane; i < M; i += 64) {
        const DevFields f = load_fields(F, d0 + i);
        t += f.tcomm;
        x += xi_term(f);
        tail += tail_term(f);
        if (f.flags & HALDA_DEV_HEAD) hi = min(hi, i);
    }
    tsum = wave_sum_f64(t);
    xsum = wave_sum_f64(x);
    tail = wave_sum_f64(tail);
    hi = wave_imin(hi);
    const int64_t h = d0 + (hi == 0x7fffffff ? 0 : hi);
    kappa = kappa_head(Mo, F.flags[h], F.scpu_b1[h], F.T_cpu[h], F.s_disk[h]) + tail;
}

// A uniform read of read-only memory through the scalar cache (s_load): the constant address space
// tells the compiler the value cannot change under the kernel (a plain global read of a uniform
// address is a vector load, a full memory round trip before the loads that depend on it).
__device__ inline int64_t sload_i64(const int64_t *p) {
    return *reinterpret_cast<const __attribute__((address_space(4))) int64_t *>(
        reinterpret_cast<uintptr_t>(p));
}

// No instruction: the record's registers are redefined for the optimiser (stops loop-invariant
// hoisting of values derived from it).
__device__ inline void opaque_rec(FieldRec &r) {
    asm volatile("" : "+v"(r.alpha), "+v"(r.b), "+v"(r.p_bp), "+v"(r.p_b), "+v"(r.cst), "+v"(r.Kset), "+v"(r.Kvram),
                 "+v"(r.cls), "+v"(r.gpu));
}

// Kernel arguments. Everything a wave reads through the scalar cache comes first (six 64-B lines:
// the model, the table pointers, the result pointers, the counts); the k list, which lanes read
// with vector loads, last.
// halda_fleet_result without x_off (ABI 2's compact layout travels at the end of SweepArgs): the
// result pointers stay within the kernel arguments' first lines, read through the scalar cache.
struct FleetOut {
    int32_t *best_k;
    double *obj_value;
    int32_t *w, *n;
    double *obj_by_k;
    int32_t *status;
    double *x, *c;
    FleetOut() = default;
    __host__ __device__ FleetOut(const halda_fleet_result &r)
        : best_k(r.best_k), obj_value(r.obj_value), w(r.w), n(r.n), obj_by_k(r.obj_by_k), status(r.status), x(r.x),
          c(r.c) {}
};

struct SweepArgs {
    halda_model Mo;
    halda_fleets F;
    int n_k;
    int uM;                        // > 0: every fleet has uM devices (dev_off[f] = dev_off[0] + f uM)
    FleetOut out;
    int64_t xstride;
    uint8_t *fflag;  // per fleet: 1 = needs the table launch
    int *hb_flag;
    int launch_id;
    int want;                      // 0: every fleet, 1: flagged fleets (gated on hb_flag)
    int k1dp;                      // register sweep: 1 = every k = 1 / W = M instance by k1_dp (test path)
    int xz;                        // 1: x / c of non-optimal instances written as zeros; 0: left as they are
                                   // (the host zero-copy path zero-fills them on the host)
    int mmax, r1max, tab, tab_kc;  // table slice shape (kTables)
    unsigned char *gtab;           // kGlobal: per-wave slices
    int64_t gstride;
    const int64_t *x_off;          // halda_fleet_result.x_off (compact x / c layout) or nullptr
    int32_t ks[64];  // the k list travels in the kernel arguments (no copy)
    int32_t Ws[64];  // W = L / k per k (host integer division)
};

// x / c of one (fleet, k) solution (col layout [w|n|s1|s2|s3|t|z|C] with the fleet's M), written
// by the lane of each device when the caller asked for them.
// Element offset of instance inst's x / c: the dense layout, or the caller's compact x_off (-1: not
// written).
__device__ inline int64_t xc_at(const SweepArgs &A, int64_t inst) {
    return A.x_off ? A.x_off[inst] : inst * A.xstride;
}

__device__ inline void put_xc(const SweepArgs &A, int64_t inst, int M, int i, int wl, int n, const int s[4], double z,
                              const FieldRec &r) {
    if (!A.out.x && !A.out.c) return;
    const int64_t at = xc_at(A, inst);
    if (at < 0) return;
    const Dev d = r.dev();
    if (A.out.x) {
        double *x = A.out.x + at;
        x[i] = double(wl); x[M + i] = double(n);
        x[2 * M + i] = double(s[0]); x[3 * M + i] = double(s[1]); x[4 * M + i] = double(s[2]);
        x[5 * M + i] = double(s[3]); x[6 * M + i] = z;
    }
    if (A.out.c) {
        double *c = A.out.c + at;
        c[i] = d.cw; c[M + i] = d.cn; c[2 * M + i] = d.cs0; c[3 * M + i] = d.cs1; c[4 * M + i] = d.cs2;
        c[5 * M + i] = d.cs3; c[6 * M + i] = 0.0;
    }
}

#ifndef HALDA_SWEEP_TABLE_K1
#define HALDA_SWEEP_TABLE_K1 1  // table launches also run the k = 1 register greedy (else k = 1 via tables)
#endif

__device__ inline void flag_fleet(const SweepArgs &A, int f, int lane) {
    // the scratch-free register launch (fflag == nullptr) never flags: sweep_fleets runs it alone only
    // when nothing in the batch can need the table launch (no k > 1 with W >= M, R + 1 <= kDpLanes)
    if (lane == 0 && A.fflag) {
        A.fflag[f] = 1;
        __hip_atomic_store(A.hb_flag, A.launch_id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// SG = Wave: one fleet per wave; SG = Seg<16>: one fleet (M <= 16, n_k <= 16) per 16-lane segment,
// tables in the segment's LDS slice, k = 1 register greedy and k > 1 incremental threshold scan
// only: what that cannot do (fast-path fallbacks, non-convex / non-monotone leaves) is flagged for
// the one-fleet-per-wave table launch, as the register-only launch does.
template <bool kTables, bool kGlobal, class SG = Wave, bool kPre = false>
__device__ void sweep_fleet(const SweepArgs &A, int f, const WaveCtx &w, const SG &sg, const DevFields &pre = {},
                            int64_t pre_base = 0) {
    constexpr int S = SG::S;
    constexpr bool kSeg = S < 64;
    constexpr bool kFirst = !kTables || kSeg;  // a first launch: flags what it leaves to the table launch
    const int lane = sg.sl;  // device index within the fleet
    const halda_model &Mo = A.Mo;
    const halda_fleets &F = A.F;
    HALDA_SSTAMP(0, __builtin_amdgcn_s_memtime());
    HALDA_SSTAMP(7, __builtin_amdgcn_s_memrealtime());
    // lane j: k_j and W_j = L / k_j (kernel arguments; their loads are issued with the fields')
    const bool kl = lane < A.n_k;
    const int kj = A.ks[kl ? lane : 0];
    const int Wj = kl ? A.Ws[lane] : 0;
    // the fleet's extent: with one fleet size for the batch, from dev_off[0] read through the scalar
    // cache (the table is read-only to the kernel), so that the field loads are the wave's first
    // vector round trip
    // with one fleet size for the batch the first device is dev_off[0] + f uM; dev_off[0] (0 in the
    // usual table) is read beside the field loads below, not in front of them
    int64_t d0 = A.uM > 0 ? int64_t(f) * A.uM : F.dev_off[f];
    const int M = A.uM > 0 ? A.uM : int(F.dev_off[f + 1] - d0);
    bool regs = M <= kK1MaxM;  // lane = device: the k = 1 greedy runs in registers
    if constexpr (kSeg) regs = true;  // the host sends fleets of at most S devices
    FieldRec me = {};
    int bad = 0;
    double tsum = 0.0, xsum = 0.0, kappa = 0.0;
    if (regs) {
        // every field of this lane's device in one round trip (lanes past M read device 0). With one
        // fleet size the loads are issued at once from dev_off[0] = 0 (the usual table) while the
        // scalar read of dev_off[0] is in flight, and reissued only where it is not 0: no dependent
        // round trip in front of the field loads.
        // pre: the caller loaded this lane's fields already (the pipelined kernel, one fleet size, its
        // dev_off[0] = pre_base applied)
        DevFields mf;
        if constexpr (kPre) mf = pre;
        else mf = load_fields(F, d0 + (lane < M ? lane : 0));
        if constexpr (kPre) {
            d0 += pre_base;
        } else if (A.uM > 0) {
            // a vector read (returns in order behind the field loads: no wait of its own, unlike a
            // scalar read, whose lgkmcnt wait would also hold the kernel-argument reads)
            const int64_t base = __builtin_amdgcn_readfirstlane(int(F.dev_off[0])) |
                                 (int64_t(__builtin_amdgcn_readfirstlane(int(uint64_t(F.dev_off[0]) >> 32))) << 32);
            if (base != 0) {
                d0 += base;
                mf = load_fields(F, d0 + (lane < M ? lane : 0));
            }
        }
#if defined(HALDA_DIAG_EXIT) && HALDA_DIAG_EXIT == 3  // diagnostic build only: the field loads alone
        if (lane < M)
            A.out.n[d0 + lane] = int(mf.scpu + mf.sgpu + mf.Tc + mf.Tg + mf.tkc + mf.tkg + mf.r2v + mf.v2r + mf.tcomm +
                                     mf.sdisk) + int(mf.ram + mf.ccpu + mf.cgpu + mf.cuda + mf.metal + mf.swap) + mf.cls + mf.flags;
        return;
#endif
        me = field_rec(Mo, mf, bad);
        bad = lane < M ? bad : 0;
        if (M > 0) fleet_offsets_regs(Mo, mf, M, sg, tsum, xsum, kappa);
    } else {
        if (A.uM > 0) d0 += sload_i64(F.dev_off);
        for (int i = lane; i < M; i += 64) {
            int b1 = 0;
            field_rec(Mo, load_fields(F, d0 + i), b1);
            bad |= b1;
        }
        fleet_offsets_tree(Mo, F, d0, M, lane, tsum, xsum, kappa);
    }
    bad = sg.any(bad != 0) ? 1 : 0;
    HALDA_SSTAMP(1, __builtin_amdgcn_s_memtime());
    HALDA_SSTAMP(9, __builtin_amdgcn_s_memrealtime());
#if defined(HALDA_DIAG_EXIT) && HALDA_DIAG_EXIT == 1  // diagnostic build only: stop after the records
    if (lane < M) A.out.n[d0 + lane] = me.Kset + me.Kvram + int(me.alpha + me.b + me.p_bp + me.p_b + me.cst) + bad + kj + Wj;
    if (lane == 0) A.out.obj_value[f] = tsum + xsum + kappa;
    return;
#endif
    double best = kInf;
    int best_k = 0;
    // the k's settled without a solve (the screen's verdicts: W >= 1e6 unsupported, M > W
    // bound-infeasible, rows decode rejects) are written lane-parallel, and the loop below visits only
    // the others, in ascending k
    constexpr int kOpen = 1000;
    int stj = kOpen;
    if (!(Wj < 1000000)) stj = HALDA_STATUS_UNSUPPORTED;
    else if (M > Wj) stj = HALDA_STATUS_INFEASIBLE;  // sum lb(w) = M > W (HiGHS presolve)
    else if (M > 0 && bad) stj = HALDA_STATUS_UNSUPPORTED;
    if (kl && stj != kOpen) {
        const int64_t inst = int64_t(f) * A.n_k + lane;
        if (A.out.obj_by_k) A.out.obj_by_k[inst] = kInf;
        if (A.out.status) A.out.status[inst] = stj;
    }
    if (A.xz && (A.out.x || A.out.c)) {  // x / c of a settled instance are zero
        uint64_t settled = sg.bits(kl && stj != kOpen);
        const int N = 7 * M + 1;
        while (settled) {
            const int j = __builtin_ctzll(settled);
            settled &= settled - 1;
            const int64_t at = xc_at(A, int64_t(f) * A.n_k + j);
            if (at >= 0)
                for (int cc = lane; cc < N; cc += S) {
                    if (A.out.x) A.out.x[at + cc] = 0.0;
                    if (A.out.c) A.out.c[at + cc] = 0.0;
                }
        }
    }
    uint64_t todo = sg.bits(kl && stj == kOpen);
    const int M_all = M;
    while (todo) {
        const int j = __builtin_ctzll(todo);
        todo &= todo - 1;
        // the record and M are opaque to the compiler at each k: nothing derived from them is hoisted
        // out of this loop (hoisted per-lane masks and addresses held across the loop spill SGPRs; most
        // fleets open one k)
        opaque_rec(me);
        int M = M_all;
        if constexpr (!kSeg) asm volatile("" : "+s"(M));
        const int k = sg.bcast(kj, j);
        const int W = sg.bcast(Wj, j);
        const int64_t inst = int64_t(f) * A.n_k + j;
        const double kc = double(k - 1);
        int st;
        double obj = kInf;
        bool improved = false;
        if (M == 0) st = W > 0 ? HALDA_STATUS_INFEASIBLE : HALDA_STATUS_OPTIMAL;  // x = [C = 0]
        else {
            int rc = K1_FALLBACK, e = 0, rounds = 0, nE = 0;
            double gE = 0.0;
            bool haveE = true;  // gE / nE hold the split at w = 1 + e (k1_alloc), else split here
            me.W = W;
            if (k == 1) HALDA_SSTAMP(2, __builtin_amdgcn_s_memtime());
#if defined(HALDA_DIAG_EXIT) && HALDA_DIAG_EXIT == 4  // diagnostic build only: stop before the first greedy
            if (lane < M) A.out.n[d0 + lane] = me.Kset + me.Kvram + int(me.alpha + me.b + me.p_bp + me.p_b + me.cst) + W + k;
            if (lane == 0) A.out.obj_value[f] = tsum + xsum + kappa;
            return;
#endif
            // k = 1: the register greedy; W = M (R = 0): every w_i = 1 is forced, so the same code gives
            // the solution for any k (the output adds (k - 1) max_i H_i)
            if ((k == 1 || W == M) && regs && (!kTables || HALDA_SWEEP_TABLE_K1 || W == M)) {
                if constexpr (!kTables) {
                    // the register launch solves its greedy fallbacks itself (exact DP, R + 1 <= kDpLanes)
                    if (!A.k1dp) rc = k1_alloc(me, M, W - M, sg, e, rounds, gE, nE);
                    if (rc == K1_FALLBACK && W - M < kDpLanes) {
                        rc = k1_dp(me, M, W - M, sg, e, w.dparg);
                        haveE = false;
                    }
                } else {
                    rc = k1_alloc(me, M, W - M, sg, e, rounds, gE, nE);
                }
            }
            if (k == 1) HALDA_SSTAMP(3, __builtin_amdgcn_s_memtime());
#if defined(HALDA_DIAG_EXIT) && HALDA_DIAG_EXIT == 2  // diagnostic build only: stop after the first greedy
            if (lane < M) A.out.n[d0 + lane] = e + rc + rounds;
            if (lane == 0) A.out.obj_value[f] = tsum + xsum + kappa;
            return;
#endif
            if (rc == K1_INFEASIBLE) {
                st = HALDA_STATUS_INFEASIBLE;
            } else if (rc == K1_OK) {
                double g = 0.0, H = 0.0, z = 0.0;
                int n = 0, sl[4] = {0, 0, 0, 0};
                const int wl = 1 + e;
                // the cycle times only matter through (k - 1) max H and the x output: at k = 1 without x
                // the largest cycle time is not formed (kc * hmax is +0 either way: hmax is finite and
                // >= 0 after a successful split)
                const bool need_h = kc != 0.0 || A.out.x;
                if (lane < M) {
                    if (haveE) {
                        g = gE;
                        n = nE;
                        rec_slacks(me, wl, n, sl);
                    } else {
                        split_full(me, wl, g, n, sl);
                    }
                    if (need_h) {
                        double P, Q;
                        dev_cycle(me, wl, n, sl, P, Q);
                        z = Q > P ? 0.5 * (Q - P) : 0.0;
                        H = Q >= P ? 0.5 * (P + Q) : P;
                    }
                }
                const double hmax = need_h ? fmax(0.0, sg.max_f64(lane < M ? H : 0.0)) : 0.0;
                obj = sg.sum_f64(lane < M ? g : 0.0) + kc * hmax;
                obj = obj + tsum;
                obj = obj + xsum;
                obj = obj + kappa;
                st = HALDA_STATUS_OPTIMAL;
                improved = obj < best;
                if (lane < M) {
                    put_xc(A, inst, M, lane, wl, n, sl, z, me);
                    if (improved) {
                        A.out.w[d0 + lane] = wl;
                        A.out.n[d0 + lane] = n;
                    }
                }
                if (lane == 0 && (A.out.x || A.out.c)) {
                    const int64_t at = xc_at(A, inst);
                    if (at >= 0 && A.out.x) A.out.x[at + 7 * M] = hmax;
                    if (at >= 0 && A.out.c) A.out.c[at + 7 * M] = kc;
                }
                HALDA_SSTAMP(4, __builtin_amdgcn_s_memtime());
            } else if constexpr (!kTables) {
                // k > 1, a wide fleet or a fast-path fallback: the table launch redoes this fleet
                flag_fleet(A, f, lane);
                return;
            } else {
                if (kSeg && (kc == 0.0 || M < 2)) {  // a k = 1 fast-path fallback / one device: the 64-lane kernel
                    flag_fleet(A, f, lane);
                    return;
                }
                Inst I = {};
                I.inst = int(inst);
                HALDA_TSTAMP(0);
                I.M = M;
                I.W = W;
                I.Wd = double(W);
                I.kc = kc;
                I.iC = 7 * M;
                I.R1 = W - M + 1;
                I.RS = odd_stride(I.R1);
                const FieldSrc src{&A.Mo, &A.F, regs ? &me : nullptr, d0, W, sg.base};
                int64_t nodes = 0;
                const bool too_large =
                    M > A.mmax || I.R1 > A.r1max || int64_t(M) * I.RS > (kc > 0.0 ? A.tab_kc : A.tab);
                if (kSeg && too_large) {
                    flag_fleet(A, f, lane);
                    return;
                }
                int feas = 1;
                if (!too_large) {
                    table_pass<S>(src, w, I, lane);
                    wave_sync();
                    HALDA_TSTAMP(6);
                    if constexpr (kSeg) {
                        feas = dp_pass_lanes(w, I, sg, nodes);
                        if (feas < 0) {  // a leaf the incremental scan does not take
                            flag_fleet(A, f, lane);
                            return;
                        }
                    } else {
                        feas = dp_pass(w, I, lane, nodes) ? 1 : 0;
                    }
                }
                if (too_large) {
                    st = HALDA_STATUS_TOO_LARGE;  // beyond the launch's slice (the host sizes it from the fleets)
                } else if (!feas) {
                    st = HALDA_STATUS_INFEASIBLE;
                } else {
                    HALDA_TSTAMP(7);
                    // solution: per device (w, n, least slacks, z), sum of costs, largest cycle time
                    double gs = 0.0, hmax = 0.0;
                    for (int i0 = 0; i0 < M; i0 += S) {
                        const int i = i0 + lane;
                        FieldRec d;
                        src.load(d, w, min(i, M - 1));
                        if (i < M) {
                            const int wl = 1 + w.st0[i];
                            double g = 0.0, P, Q;
                            int n = 0, sl[4] = {0, 0, 0, 0};
                            split_full(d, wl, g, n, sl);
                            dev_cycle(d, wl, n, sl, P, Q);
                            gs += g;
                            hmax = fmax(hmax, Q >= P ? 0.5 * (P + Q) : P);
                            put_xc(A, inst, M, i, wl, n, sl, Q > P ? 0.5 * (Q - P) : 0.0, d);
                        }
                    }
                    hmax = sg.max_f64(hmax);
                    obj = sg.sum_f64(gs) + kc * hmax;
                    obj = obj + tsum;
                    obj = obj + xsum;
                    obj = obj + kappa;
                    st = HALDA_STATUS_OPTIMAL;
                    improved = obj < best;
                    if (improved)
                        for (int i0 = 0; i0 < M; i0 += S) {
                            const int i = i0 + lane;
                            FieldRec d;
                            src.load(d, w, min(i, M - 1));
                            if (i < M) {
                                const int wl = 1 + w.st0[i];
                                double g;
                                int n = 0, sl[4];
                                split_full(d, wl, g, n, sl);
                                A.out.w[d0 + i] = wl;
                                A.out.n[d0 + i] = n;
                            }
                        }
                    if (lane == 0 && (A.out.x || A.out.c)) {
                        const int64_t at = xc_at(A, inst);
                        if (at >= 0 && A.out.x) A.out.x[at + 7 * M] = hmax;
                        if (at >= 0 && A.out.c) A.out.c[at + 7 * M] = kc;
                    }
                    HALDA_TSTAMP(8);
                }
                wave_sync();  // tables / st0 are rewritten by the next k
            }
        }
        if (st == HALDA_STATUS_OPTIMAL && M == 0) {
            obj = 0.0;  // c.x = 0; no devices: the offsets are empty sums and kappa is undefined
            improved = obj < best;
            if (lane == 0 && (A.out.x || A.out.c)) {
                const int64_t at = xc_at(A, inst);
                if (at >= 0 && A.out.x) A.out.x[at] = 0.0;
                if (at >= 0 && A.out.c) A.out.c[at] = kc;
            }
        }
        if (improved) {
            best = obj;
            best_k = k;
        }
        if (A.xz && st != HALDA_STATUS_OPTIMAL) {  // x / c of a non-optimal instance are zero
            const int N = 7 * M + 1;
            const int64_t at = xc_at(A, inst);
            if (at >= 0)
                for (int cc = lane; cc < N; cc += S) {
                    if (A.out.x) A.out.x[at + cc] = 0.0;
                    if (A.out.c) A.out.c[at + cc] = 0.0;
                }
        }
        if (lane == 0) {
            if (A.out.obj_by_k) A.out.obj_by_k[inst] = st == HALDA_STATUS_OPTIMAL ? obj : kInf;
            if (A.out.status) A.out.status[inst] = st;
        }
    }
    HALDA_SSTAMP(5, __builtin_amdgcn_s_memtime());
    if (lane == 0) {
        A.out.best_k[f] = best_k;
        A.out.obj_value[f] = best;
        if (kFirst && A.fflag) A.fflag[f] = 0;
    }
    if (best_k == 0)
        for (int i = lane; i < M; i += S) {
            A.out.w[d0 + i] = 0;
            A.out.n[d0 + i] = 0;
        }
    HALDA_SSTAMP(6, __builtin_amdgcn_s_memtime());
    HALDA_SSTAMP(8, __builtin_amdgcn_s_memrealtime());
}

template <bool kTables, bool kGlobal>
__device__ inline void sweep_body(const SweepArgs &A, unsigned char *slice_base) {
    const int lane = threadIdx.x;
    if (A.want == 1 && __hip_atomic_load(A.hb_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != A.launch_id)
        return;
    WaveCtx w = {};
    if constexpr (kTables) {
        const Slice sl = make_slice(A.mmax, A.r1max, A.tab, A.tab_kc);
        unsigned char *base = slice_base;
        w.rows = reinterpret_cast<int2 *>(base + sl.rows);
        w.cyc = reinterpret_cast<double *>(base + sl.cyc);
        w.cost = reinterpret_cast<double *>(base + sl.cost);
        w.cnt = reinterpret_cast<int *>(base + sl.cnt);
        w.st0 = reinterpret_cast<int *>(base + sl.st0);
        w.st1 = reinterpret_cast<int *>(base + sl.st1);
        w.rng = reinterpret_cast<int2 *>(base + sl.rng);
        w.inc = reinterpret_cast<double *>(base + sl.inc);
        w.G = reinterpret_cast<double *>(base + sl.G);
        w.H = reinterpret_cast<double *>(base + sl.H);
        w.work = reinterpret_cast<double *>(base + sl.work);
        w.split = reinterpret_cast<uint16_t *>(base + sl.split);
    }
    const int S = gridDim.x;
    const int nf = A.F.n_fleets;
    for (int64_t b = blockIdx.x; b < nf; b += int64_t(64) * S) {
        const int64_t mine = b + int64_t(lane) * S;
        uint64_t todo = __ballot(mine < nf && (A.want == 0 || A.fflag[mine] == 1));
        while (todo) {
            const int bit = __builtin_ctzll(todo);
            todo &= todo - 1;
            sweep_fleet<kTables, kGlobal>(A, int(b + int64_t(bit) * S), w, Wave(lane));
        }
    }
}

#ifndef HALDA_SWEEP_WAVES_PER_SIMD
#define HALDA_SWEEP_WAVES_PER_SIMD 4  // occupancy target of the register-only sweep (as the k = 1 kernel)
#endif
#ifndef HALDA_SWEEP_WPB
#define HALDA_SWEEP_WPB 4
#endif
constexpr int kSweepWavesPerBlock = HALDA_SWEEP_WPB;  // fleets per workgroup of the register-only sweep

// The register-only sweep: exactly one fleet per wave, kSweepWavesPerBlock waves per workgroup (a
// quarter of the workgroups to dispatch); no loop, so no kernel argument stays live past its use.
__global__ __launch_bounds__(64 * kSweepWavesPerBlock, HALDA_SWEEP_WAVES_PER_SIMD) void halda_sweep_kernel(SweepArgs A) {
    // wave-uniform by construction; readfirstlane lets the compiler know (scalar fleet addressing)
    const int f = __builtin_amdgcn_readfirstlane(int(blockIdx.x) * kSweepWavesPerBlock + int(threadIdx.x >> 6));
    {
        // the kernel arguments the first branches read, fetched together with one value of every other
        // 64-B line of SweepArgs the wave reads through the scalar cache (the model, the table and
        // result pointers): one round trip instead of one per branch and line (each lgkmcnt wait would
        // otherwise hold the next read back)
        const int nf = A.F.n_fleets, nk = A.n_k, um = A.uM;
        const int64_t *doff = A.F.dev_off;
        const double bp = A.Mo.b_prime;
        const double *tc = A.F.T_cpu;
        const int32_t *ow = A.out.w;
        asm volatile("" ::"s"(nf), "s"(nk), "s"(um), "s"(doff), "s"(bp), "s"(tc), "s"(ow));
    }
    if (f >= A.F.n_fleets) return;
#if defined(HALDA_DIAG_EXIT) && HALDA_DIAG_EXIT == 5  // diagnostic build only: the launch alone
    if ((threadIdx.x & 63) == 0) A.out.best_k[f] = 0;
    return;
#endif
#ifdef HALDA_SWEEP_STAGGER
    {  // experiment: the waves sharing a SIMD start their loads one after another (slot = HW wave id)
        const int slot = __builtin_amdgcn_s_getreg(4 | (3 << 11)) & 3;
        for (int q = 0; q < slot; ++q) __builtin_amdgcn_s_sleep(HALDA_SWEEP_STAGGER);
    }
#endif
    __shared__ uint8_t dparg[kSweepWavesPerBlock][64 * kDpLanes];
    WaveCtx w = {};
    w.dparg = dparg[threadIdx.x >> 6];
    sweep_fleet<false, false>(A, f, w, Wave(int(threadIdx.x & 63)));
}

// The register-only sweep, pipelined: a grid of nw waves (fewer than the fleets), wave w takes fleets
// w, w + nw, w + 2 nw, ... and issues the field loads of its next fleet before it solves the current
// one, so the next fleet's memory round trip hides behind this fleet's compute and the dispatcher
// launches nw waves instead of one per fleet. One fleet size for the batch (uM <= 64), else the
// one-fleet-per-wave kernel runs. The per-fleet work is sweep_fleet's, bit for bit.
__global__ __launch_bounds__(64 * kSweepWavesPerBlock, HALDA_SWEEP_WAVES_PER_SIMD) void halda_sweep_pipe_kernel(
    SweepArgs A, int nw) {
    const int wv = __builtin_amdgcn_readfirstlane(int(blockIdx.x) * kSweepWavesPerBlock + int(threadIdx.x >> 6));
    {
        const int nf = A.F.n_fleets, nk = A.n_k, um = A.uM;
        const int64_t *doff = A.F.dev_off;
        const double bp = A.Mo.b_prime;
        const double *tc = A.F.T_cpu;
        const int32_t *ow = A.out.w;
        asm volatile("" ::"s"(nf), "s"(nk), "s"(um), "s"(doff), "s"(bp), "s"(tc), "s"(ow));
    }
    const int nf = A.F.n_fleets;
    if (wv >= nf) return;
    const int lane = threadIdx.x & 63;
    const int M = A.uM;
    const int li = lane < M ? lane : 0;
    __shared__ uint8_t dparg[kSweepWavesPerBlock][64 * kDpLanes];
    WaveCtx w = {};
    w.dparg = dparg[threadIdx.x >> 6];
    // the first fleet's fields from dev_off[0] = 0 (the usual table), reloaded where it is not 0
    DevFields nxt = load_fields(A.F, int64_t(wv) * M + li);
    const int64_t base = __builtin_amdgcn_readfirstlane(int(A.F.dev_off[0])) |
                         (int64_t(__builtin_amdgcn_readfirstlane(int(uint64_t(A.F.dev_off[0]) >> 32))) << 32);
    if (base != 0) nxt = load_fields(A.F, base + int64_t(wv) * M + li);
    for (int f = wv; f < nf; f += nw) {
        const DevFields cur = nxt;
        const int fn = f + nw;
        if (fn < nf) nxt = load_fields(A.F, base + int64_t(fn) * M + li);  // in flight during this fleet
        sweep_fleet<false, false, Wave, true>(A, f, w, Wave(lane), cur, base);
    }
}

__global__ __launch_bounds__(64, HALDA_SOLVE_WAVES_PER_SIMD) void halda_sweep_tables_kernel(SweepArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    sweep_body<true, false>(A, smem);
}

__global__ __launch_bounds__(64, HALDA_SOLVE_WAVES_PER_SIMD) void halda_sweep_big_kernel(SweepArgs A) {
    sweep_body<true, true>(A, A.gtab + int64_t(blockIdx.x) * A.gstride);
}

// halda_sweep_seg_kernel: fleets of at most kSegLanes devices (C2: 16) with at most kSegLanes
// k-candidates, 64 / kSegLanes fleets per wave, one per lane segment, each with an LDS slice of only
// what the lane-parallel path touches: G and H (k > 1 tables, row stride RS) and st0. Every wave
// reduction of the one-fleet-per-wave path becomes a segment butterfly (same order of additions:
// the wave butterfly's first two steps only add zeros for M <= 16), so the results are the same
// bits; what the segment path does not take is flagged for the gated halda_sweep_tables_kernel.
constexpr int kSegLanes = 16;

__host__ __device__ inline int64_t seg_slice_bytes(int mmax, int tab_kc) {
    return 2 * align16(int64_t(tab_kc) * 8) + align16(int64_t(mmax) * 4);
}

#ifndef HALDA_SEG_WAVES_PER_SIMD
#define HALDA_SEG_WAVES_PER_SIMD 2
#endif

__global__ __launch_bounds__(64, HALDA_SEG_WAVES_PER_SIMD) void halda_sweep_seg_kernel(SweepArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int kPer = 64 / kSegLanes;
    const int lane = threadIdx.x;
    const Seg<kSegLanes> sg(lane);
    const int seg = lane / kSegLanes;
    const int64_t tb = align16(int64_t(A.tab_kc) * 8);
    unsigned char *base = smem + int64_t(seg) * seg_slice_bytes(A.mmax, A.tab_kc);
    WaveCtx w = {};
    w.G = reinterpret_cast<double *>(base);
    w.H = reinterpret_cast<double *>(base + tb);
    w.st0 = reinterpret_cast<int *>(base + 2 * tb);
    const int nf = A.F.n_fleets;
    for (int64_t b = int64_t(blockIdx.x) * kPer; b < nf; b += int64_t(gridDim.x) * kPer) {
        const int64_t f = b + seg;
        if (f < nf) sweep_fleet<true, false, Seg<kSegLanes>>(A, int(f), w, sg);
    }
}

// halda_sweep_kslot_kernel: the k-sweep of fleets of at most kSegLanes devices (C2) with the k's
// spread over waves. A workgroup holds four fleets (one per 16-lane segment, as the segment kernel)
// and one wave per open k-slot (the k's some fleet of the batch can take: L / k >= min_devices,
// L / k < 1e6, ascending); wave q solves k-slot q of its four fleets -- the k = 1 register greedy,
// the forced W = M split, or the k > 1 tables + threshold scan in its own LDS slice -- and leaves its
// objective, status and (w, n) in the workgroup's pick area. After one barrier, wave 0 picks each
// fleet's best k by the reference's rule (ascending k, strict "<" on obj_value,
// halda_p_solver.py:407) and writes best_k / obj_value / w / n; the k's no slot takes (settled for
// every fleet: M > W or W >= 1e6) are written there too. Same per-(fleet, k) arithmetic as
// sweep_fleet on Seg<16> (the same records, reductions and tie rules: the same bits), but the
// segment kernel's one wave per four fleets becomes one wave per (four fleets, k): four to sixteen
// times the waves to hide the reductions' and LDS round trips' latency. What the slot waves cannot
// take (greedy fallbacks, tables beyond the slice, non-convex leaves) flags the fleet for the gated
// table launch, which redoes it whole.
constexpr int kMaxSlots = 16;
constexpr int kSlotFlagged = 1000;  // SlotPick.st: the fleet goes to the table launch

struct SlotPick {  // one (segment, k-slot) result in the workgroup's pick area
    double obj;    // obj_value when OPTIMAL, else +inf
    int st;        // HALDA_STATUS_* or kSlotFlagged
    int pad;
    int w[kSegLanes], n[kSegLanes];
};

struct SlotArgs {
    int n_slot;
    int pick_off;              // LDS byte offset of the pick area (SlotPick [4][n_slot])
    int j[kMaxSlots];          // k index of slot q (ascending)
    int tab[kMaxSlots];        // doubles of G (and of H) per segment: max_devices * (R + 1) + max_devices, 0: no tables
    int r1[kMaxSlots];         // largest R + 1 of slot q over the batch
    int off[kMaxSlots];        // LDS byte offset of slot q's four segment slices
};

// One (fleet, k_j) on a 16-lane segment; the result goes to *pk (segment lane 0 writes obj / st, lane i
// its w / n candidate).
__device__ void sweep_kslot(const SweepArgs &A, int f, int j, int r1cap, int tabcap, const WaveCtx &w,
                            const Seg<kSegLanes> &sg, SlotPick *pk, unsigned long long *t_rec) {
    using SG = Seg<kSegLanes>;
    constexpr int S = SG::S;
    const int lane = sg.sl;
    const halda_model &Mo = A.Mo;
    const halda_fleets &F = A.F;
    int64_t d0 = A.uM > 0 ? int64_t(f) * A.uM + F.dev_off[0] : F.dev_off[f];
    const int M = A.uM > 0 ? A.uM : int(F.dev_off[f + 1] - d0);
    const DevFields mf = load_fields(F, d0 + (lane < M ? lane : 0));
    int bad = 0;
    FieldRec me = field_rec(Mo, mf, bad);
    bad = lane < M ? bad : 0;
    double tsum, xsum, kappa;
    fleet_offsets_regs(Mo, mf, M, sg, tsum, xsum, kappa);
    const bool anybad = sg.any(bad != 0);
#ifdef HALDA_STAMPS
    *t_rec = __builtin_amdgcn_s_memtime();
#else
    (void)t_rec;
#endif
    const int k = A.ks[j], W = A.Ws[j];
    const int64_t inst = int64_t(f) * A.n_k + j;
    const double kc = double(k - 1);
    int st;
    double obj = kInf;
    int wl = 0, nl = 0;  // this lane's (w, n) in the solution
    if (!(W < 1000000)) st = HALDA_STATUS_UNSUPPORTED;
    else if (M > W) st = HALDA_STATUS_INFEASIBLE;  // sum lb(w) = M > W (HiGHS presolve)
    else if (anybad) st = HALDA_STATUS_UNSUPPORTED;
    else {
        me.W = W;
        if (k == 1 || W == M) {
            // the register greedy; W = M (R = 0): every w_i = 1 is forced
            int e = 0, rounds = 0, nE = 0;
            double gE = 0.0;
            const int rc = k1_alloc(me, M, W - M, sg, e, rounds, gE, nE);
            if (rc == K1_INFEASIBLE) {
                st = HALDA_STATUS_INFEASIBLE;
            } else if (rc == K1_OK) {
                double g = 0.0, H = 0.0, z = 0.0;
                int n = 0, sl[4] = {0, 0, 0, 0};
                wl = 1 + e;
                const bool need_h = kc != 0.0 || A.out.x;
                if (lane < M) {
                    g = gE;
                    n = nE;
                    rec_slacks(me, wl, n, sl);
                    if (need_h) {
                        double P, Q;
                        dev_cycle(me, wl, n, sl, P, Q);
                        z = Q > P ? 0.5 * (Q - P) : 0.0;
                        H = Q >= P ? 0.5 * (P + Q) : P;
                    }
                }
                const double hmax = need_h ? fmax(0.0, sg.max_f64(lane < M ? H : 0.0)) : 0.0;
                obj = sg.sum_f64(lane < M ? g : 0.0) + kc * hmax;
                obj = obj + tsum;
                obj = obj + xsum;
                obj = obj + kappa;
                st = HALDA_STATUS_OPTIMAL;
                nl = n;
                if (lane < M) put_xc(A, inst, M, lane, wl, n, sl, z, me);
                if (lane == 0 && (A.out.x || A.out.c)) {
                    const int64_t at = xc_at(A, inst);
                    if (at >= 0 && A.out.x) A.out.x[at + 7 * M] = hmax;
                    if (at >= 0 && A.out.c) A.out.c[at + 7 * M] = kc;
                }
            } else {
                st = kSlotFlagged;  // a greedy fallback: the 64-lane table launch
            }
        } else if (M < 2) {
            st = kSlotFlagged;
        } else {
            Inst I = {};
            I.inst = int(inst);
            I.M = M;
            I.W = W;
            I.Wd = double(W);
            I.kc = kc;
            I.iC = 7 * M;
            I.R1 = W - M + 1;
            I.RS = odd_stride(I.R1);
            if (M > A.mmax || I.R1 > r1cap || int64_t(M) * I.RS > tabcap) {
                st = kSlotFlagged;  // beyond the slot's slice
            } else {
                const FieldSrc src{&A.Mo, &A.F, &me, d0, W, sg.base};
                int64_t nodes = 0;
                table_pass<S>(src, w, I, lane);
                wave_sync();
                const int feas = dp_pass_lanes(w, I, sg, nodes);
                if (feas < 0) {
                    st = kSlotFlagged;  // a leaf the incremental scan does not take
                } else if (!feas) {
                    st = HALDA_STATUS_INFEASIBLE;
                } else {
                    double g = 0.0, P = 0.0, Q = 0.0, hmax = 0.0;
                    int n = 0, sl[4] = {0, 0, 0, 0};
                    if (lane < M) {
                        wl = 1 + w.st0[lane];
                        split_full(me, wl, g, n, sl);
                        dev_cycle(me, wl, n, sl, P, Q);
                        hmax = Q >= P ? 0.5 * (P + Q) : P;
                        put_xc(A, inst, M, lane, wl, n, sl, Q > P ? 0.5 * (Q - P) : 0.0, me);
                    }
                    hmax = sg.max_f64(fmax(0.0, hmax));
                    obj = sg.sum_f64(0.0 + g) + kc * hmax;  // the segment kernel's sum (0.0 + g per lane)
                    obj = obj + tsum;
                    obj = obj + xsum;
                    obj = obj + kappa;
                    st = HALDA_STATUS_OPTIMAL;
                    nl = n;
                    if (lane == 0 && (A.out.x || A.out.c)) {
                        const int64_t at = xc_at(A, inst);
                        if (at >= 0 && A.out.x) A.out.x[at + 7 * M] = hmax;
                        if (at >= 0 && A.out.c) A.out.c[at + 7 * M] = kc;
                    }
                }
            }
        }
    }
    if (st == kSlotFlagged) {
        flag_fleet(A, f, lane);
    } else {
        if (lane == 0) {
            if (A.out.obj_by_k) A.out.obj_by_k[inst] = st == HALDA_STATUS_OPTIMAL ? obj : kInf;
            if (A.out.status) A.out.status[inst] = st;
        }
        if (A.xz && st != HALDA_STATUS_OPTIMAL && (A.out.x || A.out.c)) {  // x / c of a non-optimal instance
            const int64_t at = xc_at(A, inst);
            if (at >= 0)
                for (int cc = lane; cc < 7 * M + 1; cc += S) {
                    if (A.out.x) A.out.x[at + cc] = 0.0;
                    if (A.out.c) A.out.c[at + cc] = 0.0;
                }
        }
    }
    if (lane == 0) {
        pk->obj = st == HALDA_STATUS_OPTIMAL ? obj : kInf;
        pk->st = st;
    }
    if (lane < M) {
        pk->w[lane] = wl;
        pk->n[lane] = nl;
    }
}

// The pick of one fleet (segment lanes): best k over the slots in ascending k with strict "<", the
// settled k's of no slot, best_k / obj_value / w / n and the fleet's flag byte.
__device__ void kslot_pick(const SweepArgs &A, const SlotArgs &SA, int f, const SlotPick *pk, const Seg<kSegLanes> &sg) {
    constexpr int S = kSegLanes;
    const int lane = sg.sl;
    const int64_t d0 = A.uM > 0 ? int64_t(f) * A.uM + A.F.dev_off[0] : A.F.dev_off[f];
    const int M = A.uM > 0 ? A.uM : int(A.F.dev_off[f + 1] - d0);
    bool flagged = false;
    double best = kInf;
    int bq = -1;
    for (int q = 0; q < SA.n_slot; ++q) {
        const int st = pk[q].st;
        flagged = flagged || st == kSlotFlagged;
        if (st == HALDA_STATUS_OPTIMAL && pk[q].obj < best) {
            best = pk[q].obj;
            bq = q;
        }
    }
    if (flagged) return;  // the table launch redoes this fleet (fflag / hb_flag set by the slot wave)
    // k's of no slot: settled for every fleet of the batch (W >= 1e6 unsupported, else M > W)
    for (int jj = lane; jj < A.n_k; jj += S) {
        bool slot = false;
        for (int q = 0; q < SA.n_slot; ++q) slot = slot || SA.j[q] == jj;
        if (slot) continue;
        const int64_t inst = int64_t(f) * A.n_k + jj;
        const int st = !(A.Ws[jj] < 1000000) ? HALDA_STATUS_UNSUPPORTED : HALDA_STATUS_INFEASIBLE;
        if (A.out.obj_by_k) A.out.obj_by_k[inst] = kInf;
        if (A.out.status) A.out.status[inst] = st;
        if (A.xz && (A.out.x || A.out.c)) {
            const int64_t at = xc_at(A, inst);
            if (at >= 0)
                for (int cc = 0; cc < 7 * M + 1; ++cc) {
                    if (A.out.x) A.out.x[at + cc] = 0.0;
                    if (A.out.c) A.out.c[at + cc] = 0.0;
                }
        }
    }
    if (lane == 0) {
        A.out.best_k[f] = bq >= 0 ? A.ks[SA.j[bq]] : 0;
        A.out.obj_value[f] = best;
        A.fflag[f] = 0;
    }
    if (lane < M) {
        A.out.w[d0 + lane] = bq >= 0 ? pk[bq].w[lane] : 0;
        A.out.n[d0 + lane] = bq >= 0 ? pk[bq].n[lane] : 0;
    }
}

__global__ __launch_bounds__(64 * kMaxSlots) void halda_sweep_kslot_kernel(SweepArgs A, SlotArgs SA) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int kPer = 64 / kSegLanes;
    const int lane = threadIdx.x & 63;
    const int q = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));  // this wave's k-slot
    const Seg<kSegLanes> sg(lane);
    const int seg = lane / kSegLanes;
    const int nf = A.F.n_fleets;
    const int64_t f = int64_t(blockIdx.x) * kPer + seg;
    SlotPick *pick = reinterpret_cast<SlotPick *>(smem + SA.pick_off);
    HALDA_KSTAMPW(0, __builtin_amdgcn_s_memtime());
    HALDA_KSTAMPW(5, __builtin_amdgcn_s_memrealtime());
    {
        const int tab = SA.tab[q];
        const int64_t tb = align16(int64_t(tab) * 8);
        unsigned char *base = smem + SA.off[q] + int64_t(seg) * seg_slice_bytes(A.mmax, tab);
        WaveCtx w = {};
        w.G = reinterpret_cast<double *>(base);
        w.H = reinterpret_cast<double *>(base + tb);
        w.st0 = reinterpret_cast<int *>(base + 2 * tb);
        unsigned long long t_rec = 0;
        if (f < nf) sweep_kslot(A, int(f), SA.j[q], SA.r1[q], tab, w, sg, pick + seg * SA.n_slot + q, &t_rec);
        HALDA_KSTAMPW(1, t_rec);
    }
    HALDA_KSTAMPW(2, __builtin_amdgcn_s_memtime());
    __syncthreads();
    HALDA_KSTAMPW(3, __builtin_amdgcn_s_memtime());
    if (q == 0 && f < nf) kslot_pick(A, SA, int(f), pick + seg * SA.n_slot, sg);
    HALDA_KSTAMPW(4, __builtin_amdgcn_s_memtime());
}

// halda_pick_kernel: one wave per fleet. obj_value per k = c.x + sum t_comm +
// sum xi + kappa (halda_p_solver.py:356-357), best k by ascending k with strict
// "<" (halda_p_solver.py:407), w / n of the winner (int(round(x)), :350-351).
__global__ __launch_bounds__(64) void halda_pick_kernel(halda_batch B, halda_result R, halda_fleets F, int n_k,
                                                        const double *offs, halda_fleet_result out, int64_t xstride) {
    const int lane = threadIdx.x;
    const int f = blockIdx.x;
    if (f >= F.n_fleets) return;
    int best_j = -1;
    double best = kInf;
    for (int j = 0; j < n_k; ++j) {
        const int64_t inst = int64_t(f) * n_k + j;
        const int st = R.status[inst];
        double obj = kInf;
        if (st == HALDA_STATUS_OPTIMAL) {
            const int64_t co = B.col_off[inst];
            const int N = B.n_cols[inst];
            double part = 0.0;
            for (int c = lane; c < N; c += 64) part += B.c[co + c] * R.x[co + c];
            obj = wave_sum_f64(part);
            obj = obj + offs[3 * f + 0];
            obj = obj + offs[3 * f + 1];
            obj = obj + offs[3 * f + 2];
            if (obj < best) {
                best = obj;
                best_j = j;
            }
        }
        if (lane == 0) {
            if (out.obj_by_k) out.obj_by_k[inst] = obj;
            if (out.status) out.status[inst] = st;
        }
        const int64_t at = out.x_off ? out.x_off[inst] : inst * xstride;
        if ((out.x || out.c) && at >= 0) {
            const int64_t co = B.col_off[inst];
            const int N = B.n_cols[inst];
            for (int cc = lane; cc < N; cc += 64) {
                if (out.x) out.x[at + cc] = st == HALDA_STATUS_OPTIMAL ? R.x[co + cc] : 0.0;
                if (out.c) out.c[at + cc] = st == HALDA_STATUS_OPTIMAL ? B.c[co + cc] : 0.0;
            }
        }
    }
    const int64_t d0 = F.dev_off[f];
    const int M = int(F.dev_off[f + 1] - d0);
    if (lane == 0) {
        out.best_k[f] = best_j >= 0 ? int(B.c[B.col_off[int64_t(f) * n_k + best_j] + 7 * M]) + 1 : 0;
        out.obj_value[f] = best;
    }
    for (int i = lane; i < M; i += 64) {
        int w = 0, n = 0;
        if (best_j >= 0) {
            const int64_t co = B.col_off[int64_t(f) * n_k + best_j];
            w = int(rint(R.x[co + i]));
            n = int(rint(R.x[co + M + i]));
        }
        out.w[d0 + i] = w;
        out.n[d0 + i] = n;
    }
}

// ------------------------------------------------------------------ host side
thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                                       \
    do {                                                                                                    \
        hipError_t e_ = (expr);                                                                             \
        if (e_ != hipSuccess) return fail(HALDA_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

struct Ctx {
    int device = 0;
    int cus = 256;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, evs = nullptr, evk = nullptr;  // start, end, after k = 1, after screen
    bool timed = false;
    bool timing = true;  // record the per-launch HIP events (halda_set_timing)
    bool two_pass = true;  // HALDA_TWO_PASS=0: the fused one-wave-per-instance screen + k = 1 kernel
    bool xcd_swizzle = true;  // HALDA_XCD_SWIZZLE=0: block b works on instance b
    int *hb_flag = nullptr;  // launch id of the last launch with a k = 1 hand-back
    int launch_id = 0;
    void *scratch = nullptr;  // host-API staging (device)
    void *pinned = nullptr;   // host-API staging (pinned host), one PCIe copy each way
    size_t pinned_bytes = 0;
    size_t scratch_bytes = 0;
    void *work = nullptr;  // cls[n]: screen verdict per instance
    size_t work_bytes = 0;
    void *gtab = nullptr;  // per-wave global-memory slices of the big-table general launch
    size_t gtab_bytes = 0;
    hipEvent_t ev_order = nullptr;  // cross-stream ordering of consecutive launches on this context
    hipEvent_t ev_host = nullptr;   // completion of a small synchronous call (polled, not waited on)
    hipEvent_t evf0 = nullptr, evf1 = nullptr;  // around a halda_solve_fleets sequence (lowering .. pick)
    hipEvent_t evfm = nullptr;                   // fused sweep: between its first and second launch
    bool fleet_two = false;                      // fused sweep: a second launch was enqueued
    bool fleet_reg_alone = false;                // fused sweep: the register launch alone
    bool fleet_seg = false;                      // fused sweep: the first launch was the segment kernel
    bool fleet_kslot = false;                    // fused sweep: the first launch was the k-slot kernel
    bool kslot_sweep = true;                     // fused sweep: k-slot launch where it applies (else segment)
    int sweep_waves = 0;                         // > 0: the register launch as the pipelined kernel, this many waves
    bool fleet_timed = false;
    bool fleets_fused = true;      // halda_solve_fleets: the fused sweep (default) or the CSR pipeline
    bool seg_sweep = true;         // fused sweep: lane-segment launch for fleets of <= kSegLanes devices
    bool k1_force_dp = false;      // fused sweep, test path: every register-launch k = 1 solve by k1_dp
    bool x_zero = true;            // fused sweep: x / c of non-optimal instances written as zeros
    bool last_fleet_fused = false;
    void *shard = nullptr;         // rank-local results of halda_solve_fleets_sharded
    size_t shard_bytes = 0;
    void *fflag = nullptr;         // per-fleet "needs the table launch" bytes of the fused sweep
    size_t fflag_bytes = 0;
    hipStream_t last_stream = nullptr;
    bool have_last = false;
    void *fleet_scratch = nullptr;  // lowered batch + results of halda_solve_fleets
    size_t fleet_scratch_bytes = 0;
    halda_batch last_lowered = {};
    halda_result last_solved = {};
    bool have_lowered = false;
    // resident workgroups per CU by (kernel, dynamic LDS), raising the LDS limit once per size
    struct Occ {
        const void *fn;
        int64_t lds;
        int per_cu;
    } occ[8] = {};
    int n_occ = 0;
    hipError_t occupancy(const void *fn, int64_t lds, int *per_cu) {
        for (int i = 0; i < n_occ; ++i)
            if (occ[i].fn == fn && occ[i].lds == lds) {
                if (per_cu) *per_cu = occ[i].per_cu;
                return hipSuccess;
            }
        hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
        int p = 0;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&p, fn, 64, size_t(lds));
        if (e != hipSuccess) return e;
        p = std::max(1, p);
        occ[n_occ % 8] = Occ{fn, lds, p};
        n_occ = std::min(n_occ + 1, 8);
        if (per_cu) *per_cu = p;
        return hipSuccess;
    }
};

int64_t slice_bytes_for(int mmax, int r1max, int tab, int tab_kc) {
    return make_slice(mmax, r1max, tab, tab_kc).total;
}

// On-chip budget of one general-kernel slice (LDS per CU is 160 KiB) and, for a batch whose shape
// summary exceeds it, the capped LDS slice (2 waves per CU) plus the global-table launch's HBM budget.
constexpr int64_t kLdsBudget = 160 * 1024;
constexpr int64_t kLdsCapped = 80 * 1024;
constexpr int64_t kGlobalTableBudget = int64_t(2) << 30;
constexpr int kMaxR1 = 1 << 20;  // the screen rejects W >= 1e6 anyway

struct GenShape {
    int mmax, r1, tab, tab_kc;
};

// LDS shape of the general kernel's launches for a batch summary (full when it fits the budget).
GenShape lds_shape(const GenShape &full, bool *big) {
    const int64_t need = std::max(slice_bytes_for(full.mmax, full.r1, full.tab, 0),
                                  slice_bytes_for(full.mmax, full.r1, 0, full.tab_kc));
    *big = need > kLdsBudget;
    if (!*big) return full;
    GenShape g;
    g.mmax = std::min(full.mmax, kK1MaxM);
    g.r1 = std::min(full.r1, 128);
    while (true) {
        const int t = g.mmax * odd_stride(g.r1);
        g.tab = full.tab > 0 ? std::min(full.tab, t) : 0;
        g.tab_kc = full.tab_kc > 0 ? std::min(full.tab_kc, t) : 0;
        const int64_t b = std::max(slice_bytes_for(g.mmax, g.r1, std::max(g.tab, 1), 0),
                                   slice_bytes_for(g.mmax, g.r1, 0, g.tab_kc));
        if (b <= kLdsCapped || g.r1 <= 8) break;
        g.r1 = (g.r1 + 1) / 2;
    }
    g.tab = std::max(g.tab, 1);
    return g;
}

// Device-side ordering across streams: the verdict bytes, the hand-back flag and the fleet scratch
// are per context, so a launch that uses them on another stream than the previous such launch
// waits for everything enqueued on that stream so far (same stream: stream order already
// serialises them). A launch that touches none of them (the fused sweep's register launch when it
// needs no table launch behind it) neither waits nor is waited for: independent batches on two
// streams overlap on the device.
int order_after_previous(Ctx *ctx, hipStream_t s) {
    if (ctx->have_last && ctx->last_stream != s) {
        HIP_TRY(hipEventRecord(ctx->ev_order, ctx->last_stream));
        HIP_TRY(hipStreamWaitEvent(s, ctx->ev_order, 0));
    }
    ctx->last_stream = s;
    ctx->have_last = true;
    return HALDA_OK;
}

int launch(Ctx *ctx, const halda_batch &in, const halda_result &out, hipStream_t stream) {
    if (in.n_inst <= 0) return HALDA_OK;
    if (in.max_cols < 1 || in.max_R1 < 1 || in.max_tab < 0 || in.max_tab_kc < 0)
        return fail(HALDA_E_ARG, "halda_batch shape summary (max_cols/max_R1/max_tab/max_tab_kc) not set");
    if (in.max_R1 > kMaxR1) return fail(HALDA_E_ARG, "max_R1 > 2^20 (W - sum lb(w) must be < 2^20)");
    const int mmax = (in.max_cols - 1) / 7 + 1;
    // table sizes in doubles with the odd row stride used on chip
    // M * RS <= M * (R + 1) + M: the odd row stride costs at most one double per device
    const int64_t tab = std::max<int64_t>(1, in.max_tab > 0 ? int64_t(in.max_tab) + mmax : 0);
    const int64_t tab_kc = in.max_tab_kc > 0 ? int64_t(in.max_tab_kc) + mmax : 0;
    if (tab > (1 << 27) || tab_kc > (1 << 27)) return fail(HALDA_E_ARG, "table summary out of range (> 2^27)");
    const GenShape full{mmax, in.max_R1, int(tab), int(tab_kc)};
    bool big = false;
    const GenShape ls = lds_shape(full, &big);
    const size_t n = size_t(in.n_inst);
    if (n > ctx->work_bytes) {
        if (ctx->work) HIP_TRY(hipFree(ctx->work));
        ctx->work = nullptr;
        ctx->work_bytes = 0;
        HIP_TRY(hipMalloc(&ctx->work, (n + 255) & ~size_t(255)));
        ctx->work_bytes = (n + 255) & ~size_t(255);
    }
    // global tables of the big launch: one slice per resident wave, grown on demand
    int64_t gstride = 0;
    int ggrid = 0;
    if (big) {
        gstride = (make_slice(full.mmax, full.r1, full.tab, full.tab_kc).total + 255) & ~int64_t(255);
        int per_cu = 0;
        HIP_TRY(ctx->occupancy(reinterpret_cast<const void *>(halda_solve_big_kernel), 0, &per_cu));
        ggrid = int(std::max<int64_t>(
            1, std::min<int64_t>({int64_t(ctx->cus) * per_cu, int64_t(n), kGlobalTableBudget / gstride})));
        const size_t need = size_t(gstride) * size_t(ggrid);
        if (need > ctx->gtab_bytes) {
            if (ctx->gtab) HIP_TRY(hipFree(ctx->gtab));
            ctx->gtab = nullptr;
            ctx->gtab_bytes = 0;
            HIP_TRY(hipMalloc(&ctx->gtab, need));
            ctx->gtab_bytes = need;
        }
    }
    {
        const int rc = order_after_previous(ctx, stream);
        if (rc != HALDA_OK) return rc;
    }
    uint8_t *cls = static_cast<uint8_t *>(ctx->work);
    const int launch_id = ++ctx->launch_id;  // tags this launch's k = 1 hand-backs (no reset needed)
    if (ctx->timing) HIP_TRY(hipEventRecord(ctx->ev0, stream));
    const int64_t lds1 = make_k1_slice(std::min(mmax, kK1MaxM)).total;
    if (!ctx->two_pass) {
        // one wave per instance: screen, then the k = 1 solve for the survivors
        int per_cu = 0;
        HIP_TRY(ctx->occupancy(reinterpret_cast<const void *>(halda_screen_k1_kernel), lds1, &per_cu));
        hipLaunchKernelGGL(halda_screen_k1_kernel, dim3(unsigned(in.n_inst)), dim3(64), size_t(lds1), stream, in, out,
                           cls, mmax, in.max_R1, int(tab), int(tab_kc), ctx->hb_flag, launch_id, int(ctx->xcd_swizzle));
        HIP_TRY(hipGetLastError());
        if (ctx->timing) HIP_TRY(hipEventRecord(ctx->evk, stream));
    } else {
        // two passes: screen kernel (8 instances per wave), then a persistent k = 1 kernel
        const int64_t screen_waves = (int64_t(in.n_inst) + kScreenPer - 1) / kScreenPer;
        hipLaunchKernelGGL(halda_screen_kernel, dim3(unsigned((screen_waves + 3) / 4)), dim3(256), 0, stream, in, out,
                           cls, mmax, in.max_R1, int(tab), int(tab_kc));
        HIP_TRY(hipGetLastError());
        if (ctx->timing) HIP_TRY(hipEventRecord(ctx->evk, stream));
        int per_cu = 0;
        HIP_TRY(ctx->occupancy(reinterpret_cast<const void *>(halda_solve_k1_kernel), lds1, &per_cu));
        const int grid = int(std::max<int64_t>(1, std::min<int64_t>(int64_t(ctx->cus) * per_cu, in.n_inst)));
        hipLaunchKernelGGL(halda_solve_k1_kernel, dim3(grid), dim3(64), size_t(lds1), stream, in, out, cls, mmax,
                           ctx->hb_flag, launch_id);
        HIP_TRY(hipGetLastError());
    }
    if (ctx->timing) HIP_TRY(hipEventRecord(ctx->evs, stream));
    // general kernel, two launches with their own LDS slices: k > 1 instances (tables of the k > 1
    // shape only), then k = 1 instances of fleets wider than kK1MaxM devices and the fast path's
    // hand-backs (k = 1 tables). The first runs only when the shape summary admits k > 1 instances;
    // the second is gated on the hand-back flag unless wide k = 1 fleets are possible. A batch whose
    // summary exceeds the LDS budget gets capped slices and a third launch on global-memory tables
    // for the instances beyond them.
    const bool wide = (in.max_cols - 1) / 7 > kK1MaxM;
    if (ls.tab_kc > 0) {
        const int64_t lds_kc = slice_bytes_for(ls.mmax, ls.r1, 0, ls.tab_kc);
        int per_cu = 0;
        HIP_TRY(ctx->occupancy(reinterpret_cast<const void *>(halda_solve_kernel), lds_kc, &per_cu));
        const int grid = int(std::max<int64_t>(1, std::min<int64_t>(int64_t(ctx->cus) * per_cu, in.n_inst)));
        hipLaunchKernelGGL(halda_solve_kernel, dim3(grid), dim3(64), size_t(lds_kc), stream, in, out, cls, ls.mmax,
                           ls.r1, 0, ls.tab_kc, static_cast<const int *>(ctx->hb_flag), launch_id, 0, int(CLS_GEN));
        HIP_TRY(hipGetLastError());
    }
    {
        const int64_t lds_k1 = slice_bytes_for(ls.mmax, ls.r1, ls.tab, 0);
        int per_cu = 0;
        HIP_TRY(ctx->occupancy(reinterpret_cast<const void *>(halda_solve_kernel), lds_k1, &per_cu));
        const int64_t cap = wide ? int64_t(ctx->cus) * per_cu : int64_t(ctx->cus);
        const int grid = int(std::max<int64_t>(1, std::min<int64_t>(cap, in.n_inst)));
        hipLaunchKernelGGL(halda_solve_kernel, dim3(grid), dim3(64), size_t(lds_k1), stream, in, out, cls, ls.mmax,
                           ls.r1, ls.tab, 0, static_cast<const int *>(ctx->hb_flag), launch_id, int(!wide),
                           int(CLS_GEN1));
        HIP_TRY(hipGetLastError());
    }
    if (big) {
        hipLaunchKernelGGL(halda_solve_big_kernel, dim3(unsigned(ggrid)), dim3(64), 0, stream, in, out, cls,
                           full.mmax, full.r1, full.tab, full.tab_kc, static_cast<unsigned char *>(ctx->gtab),
                           gstride);
        HIP_TRY(hipGetLastError());
    }
    if (ctx->timing) HIP_TRY(hipEventRecord(ctx->ev1, stream));
    if (ctx->timing) ctx->timed = true;
    return HALDA_OK;
}

// Fused k-sweep (halda_sweep_kernel): one register-only launch over every fleet, then the table
// launch for the fleets it flagged (gated on the hand-back flag); a batch whose k > 1 / wide
// fleets need tables from the start gets the table launch only (LDS slice), or, beyond the LDS
// budget, the register launch plus the global-table launch.
constexpr int kSweepSmallBatch = 64;

int sweep_fleets(Ctx *c, const halda_model &model, const halda_fleets &F, const int32_t *kh, int n_k,
                 const halda_fleet_result &out, hipStream_t s) {
    const int nf = F.n_fleets;
    int64_t r1_k1 = 0, r1_kc = 0;
    for (int j = 0; j < n_k; ++j) {
        const int64_t r1 = int64_t(model.L / kh[j]) - F.min_devices + 1;
        if (kh[j] == 1) r1_k1 = std::max(r1_k1, r1);
        else r1_kc = std::max(r1_kc, r1);
    }
    const int mmax = F.max_devices;
    const int64_t r1max = std::max<int64_t>(1, std::max(r1_k1, r1_kc));
    // table sizes in doubles (odd row stride: at most one extra double per device)
    const int64_t tab = r1_k1 > 0 ? int64_t(mmax) * r1_k1 + mmax : 1;
    const int64_t tab_kc = r1_kc > 0 ? int64_t(mmax) * r1_kc + mmax : 0;
    if (r1max > kMaxR1 || tab > (1 << 27) || tab_kc > (1 << 27))
        return fail(HALDA_E_ARG, "fleet shape out of range: (L / k_min - min_devices + 1) * max_devices > 2^27");
    const bool tables_first = tab_kc > 0 || mmax > kK1MaxM;
    const int64_t slice = make_slice(mmax, int(r1max), int(tab), int(tab_kc)).total;
    const bool fits = slice <= kLdsBudget;
    // fleets of <= 16 devices needing k > 1 tables: the lane-segment launch (four fleets per wave),
    // then the table launch for what it flagged
    const int64_t seg_lds = seg_slice_bytes(mmax, int(tab_kc)) * (64 / kSegLanes);
    // k-slot launch (preferred): the same fleets, one wave per (four fleets, open k)
    SlotArgs SA = {};
    int64_t kslot_lds = 0;
    for (int j = 0; j < n_k && SA.n_slot < kMaxSlots; ++j) {
        const int W = model.L / kh[j];
        if (!(W < 1000000) || W < F.min_devices) continue;  // settled for every fleet of the batch
        const int q = SA.n_slot++;
        SA.j[q] = j;
        SA.r1[q] = W - F.min_devices + 1;
        SA.tab[q] = kh[j] > 1 && W > F.min_devices ? mmax * SA.r1[q] + mmax : 0;
        SA.off[q] = int(kslot_lds);
        kslot_lds += (64 / kSegLanes) * seg_slice_bytes(mmax, SA.tab[q]);
    }
    bool kslot_all = true;  // every k that is open for some fleet has a slot
    for (int j = 0, q = 0; j < n_k; ++j) {
        const int W = model.L / kh[j];
        if (!(W < 1000000) || W < F.min_devices) continue;
        kslot_all = kslot_all && q < SA.n_slot && SA.j[q] == j;
        ++q;
    }
    SA.pick_off = int(kslot_lds);
    kslot_lds += int64_t(64 / kSegLanes) * SA.n_slot * int64_t(sizeof(SlotPick));
    const bool kslot = c->seg_sweep && c->kslot_sweep && fits && mmax <= kSegLanes && tab_kc > 0 && kslot_all &&
                       SA.n_slot >= 1 && nf > kSweepSmallBatch && kslot_lds <= kLdsBudget;
    const bool seg = !kslot && c->seg_sweep && fits && mmax <= kSegLanes && n_k <= kSegLanes && tab_kc > 0 &&
                     nf > kSweepSmallBatch && seg_lds <= kLdsBudget;
    // small batches (a single halda_solve) take one launch: the register kernel when it needs no table
    // launch behind it, else the table kernel alone
    const bool small_tables = nf <= kSweepSmallBatch && r1_k1 > kDpLanes;
    const bool reg_mode = !seg && !kslot && !(fits && (tables_first || small_tables));
    // the register launch flags k > 1 / wide fleets (tables_first) and k = 1 greedy fallbacks with
    // R + 1 > kDpLanes; the others it solves itself (k1_dp), so no table launch is needed without them
    const bool gate = tables_first || r1_k1 > kDpLanes;
    const bool scratch = !(reg_mode && !gate);  // flags / hand-back flag of this context in use
    if (scratch) {
        const int rc = order_after_previous(c, s);
        if (rc != HALDA_OK) return rc;
    }
    // staging: ks and the per-fleet flags
    const size_t need = 256 + ((size_t(nf) + 255) & ~size_t(255));
    if (need > c->fflag_bytes) {
        if (c->fflag) HIP_TRY(hipFree(c->fflag));
        c->fflag = nullptr;
        c->fflag_bytes = 0;
        HIP_TRY(hipMalloc(&c->fflag, need));
        c->fflag_bytes = need;
    }
    SweepArgs A = {};
    A.Mo = model;
    A.F = F;
    for (int j = 0; j < n_k; ++j) {
        A.ks[j] = kh[j];
        A.Ws[j] = kh[j] != 0 ? model.L / kh[j] : 0;
    }
    A.n_k = n_k;
    A.out = FleetOut(out);
    A.x_off = out.x_off;
    A.xstride = 7 * int64_t(std::max(mmax, 1)) + 1;
    A.fflag = scratch ? static_cast<uint8_t *>(c->fflag) + 256 : nullptr;
    A.hb_flag = c->hb_flag;
    A.launch_id = ++c->launch_id;
    A.mmax = mmax;
    A.uM = F.min_devices == F.max_devices ? F.max_devices : 0;
    A.k1dp = c->k1_force_dp ? 1 : 0;
    A.xz = c->x_zero ? 1 : 0;
    A.r1max = int(r1max);
    A.tab = int(tab);
    A.tab_kc = int(tab_kc);
    c->fleet_timed = false;
    c->have_lowered = false;
    if (c->timing) HIP_TRY(hipEventRecord(c->evf0, s));
    if (kslot) {
        HIP_TRY(c->occupancy(reinterpret_cast<const void *>(halda_sweep_kslot_kernel), kslot_lds, nullptr));
        const int64_t groups = (int64_t(nf) + 64 / kSegLanes - 1) / (64 / kSegLanes);
        A.want = 0;
        hipLaunchKernelGGL(halda_sweep_kslot_kernel, dim3(unsigned(groups)), dim3(64 * SA.n_slot), size_t(kslot_lds), s,
                           A, SA);
        HIP_TRY(hipGetLastError());
        if (c->timing) HIP_TRY(hipEventRecord(c->evfm, s));
        A.want = 1;
        int per_cu = 0;
        HIP_TRY(c->occupancy(reinterpret_cast<const void *>(halda_sweep_tables_kernel), slice, &per_cu));
        hipLaunchKernelGGL(halda_sweep_tables_kernel, dim3(unsigned(std::min<int64_t>(c->cus, nf))), dim3(64),
                           size_t(slice), s, A);
        HIP_TRY(hipGetLastError());
    } else if (seg) {
        int per_cu = 0;
        HIP_TRY(c->occupancy(reinterpret_cast<const void *>(halda_sweep_seg_kernel), seg_lds, &per_cu));
        const int64_t nw = (int64_t(nf) + 64 / kSegLanes - 1) / (64 / kSegLanes);
        const int grid = int(std::max<int64_t>(1, std::min<int64_t>(int64_t(c->cus) * per_cu, nw)));
        A.want = 0;
        hipLaunchKernelGGL(halda_sweep_seg_kernel, dim3(grid), dim3(64), size_t(seg_lds), s, A);
        HIP_TRY(hipGetLastError());
        if (c->timing) HIP_TRY(hipEventRecord(c->evfm, s));
        A.want = 1;
        HIP_TRY(c->occupancy(reinterpret_cast<const void *>(halda_sweep_tables_kernel), slice, &per_cu));
        hipLaunchKernelGGL(halda_sweep_tables_kernel, dim3(unsigned(std::min<int64_t>(c->cus, nf))), dim3(64),
                           size_t(slice), s, A);
        HIP_TRY(hipGetLastError());
    } else if (fits && (tables_first || small_tables)) {
        // small batches (a single halda_solve): one launch with the table slice instead of two
        int per_cu = 0;
        HIP_TRY(c->occupancy(reinterpret_cast<const void *>(halda_sweep_tables_kernel), slice, &per_cu));
        const int grid = int(std::max<int64_t>(1, std::min<int64_t>(int64_t(c->cus) * per_cu, nf)));
        A.want = 0;
        hipLaunchKernelGGL(halda_sweep_tables_kernel, dim3(grid), dim3(64), size_t(slice), s, A);
        HIP_TRY(hipGetLastError());
    } else {
        A.want = 0;
        const int pipe_waves = c->sweep_waves > 0 && A.uM > 0 && A.uM <= kK1MaxM && nf > c->sweep_waves ? c->sweep_waves : 0;
        if (pipe_waves > 0) {
            hipLaunchKernelGGL(halda_sweep_pipe_kernel,
                               dim3(unsigned((pipe_waves + kSweepWavesPerBlock - 1) / kSweepWavesPerBlock)),
                               dim3(64 * kSweepWavesPerBlock), 0, s, A, pipe_waves);
        } else {
            hipLaunchKernelGGL(halda_sweep_kernel, dim3(unsigned((nf + kSweepWavesPerBlock - 1) / kSweepWavesPerBlock)),
                               dim3(64 * kSweepWavesPerBlock), 0, s, A);
        }
        HIP_TRY(hipGetLastError());
        if (c->timing) HIP_TRY(hipEventRecord(c->evfm, s));
        A.want = 1;  // the fleets flagged above, gated on the hand-back flag
        if (!gate) {
        } else if (fits) {  // flagged fleets are rare (fast-path fallbacks): one wave per CU is plenty
            int per_cu = 0;
            HIP_TRY(c->occupancy(reinterpret_cast<const void *>(halda_sweep_tables_kernel), slice, &per_cu));
            int grid = int(std::max<int64_t>(1, std::min<int64_t>(tables_first ? int64_t(c->cus) * per_cu
                                                                             : int64_t(c->cus), nf)));
#ifdef HALDA_DIAG_GATE_GRID1
            grid = 1;  // diagnostic build only: launch cost of the gated kernel vs its grid
#endif
            hipLaunchKernelGGL(halda_sweep_tables_kernel, dim3(grid), dim3(64), size_t(slice), s, A);
        } else {
            A.gstride = (slice + 255) & ~int64_t(255);
            int per_cu = 0;
            HIP_TRY(c->occupancy(reinterpret_cast<const void *>(halda_sweep_big_kernel), 0, &per_cu));
            const int grid = int(std::max<int64_t>(
                1, std::min<int64_t>({int64_t(c->cus) * per_cu, int64_t(nf), kGlobalTableBudget / A.gstride})));
            const size_t gneed = size_t(A.gstride) * size_t(grid);
            if (gneed > c->gtab_bytes) {
                if (c->gtab) HIP_TRY(hipFree(c->gtab));
                c->gtab = nullptr;
                c->gtab_bytes = 0;
                HIP_TRY(hipMalloc(&c->gtab, gneed));
                c->gtab_bytes = gneed;
            }
            A.gtab = static_cast<unsigned char *>(c->gtab);
            hipLaunchKernelGGL(halda_sweep_big_kernel, dim3(grid), dim3(64), 0, s, A);
        }
        HIP_TRY(hipGetLastError());
    }
    if (c->timing) {
        HIP_TRY(hipEventRecord(c->evf1, s));
        c->fleet_timed = true;
    }
    c->fleet_two = seg || kslot || (reg_mode && gate);
    c->fleet_reg_alone = reg_mode && !gate;
    c->fleet_seg = seg;
    c->fleet_kslot = kslot;
    c->last_fleet_fused = true;
    return HALDA_OK;
}

// ---------------------------------------------------------------- latency mode over RCCL
// One process per GPU, the ranks of an RCCL communicator: rank r sweeps the k-candidates
// ks[r], ks[r + world], ... of every fleet (halda_sweep_* on its own GPU), then the ranks agree on each
// fleet's best k with the reference's rule -- the smallest obj_value, ties to the smallest k
// (halda_p_solver.py:407) -- by three all-reduces over xGMI: MIN of obj_value, MIN of the k that
// reaches it, SUM of (w, n) where only the owner of that k contributes (the ranks' k's are disjoint),
// plus MIN / MAX of the per-k objectives / statuses when requested. Kernels between them turn one
// reduction's output into the next one's input on the device; nothing returns to the host.
__global__ __launch_bounds__(64) void halda_shard_kernel(int mode, int n_k, int n_sub, int rank, int world,
                                                         const int64_t *dev_off, halda_fleet_result sub,
                                                         halda_fleet_result out) {
    const int f = blockIdx.x, lane = threadIdx.x;
    const int64_t d0 = dev_off[f], d1 = dev_off[f + 1];
    if (mode == 0) {  // local results into the full layout, neutral elements elsewhere
        if (lane == 0) out.obj_value[f] = n_sub > 0 ? sub.obj_value[f] : kInf;
        for (int64_t d = d0 + lane; d < d1; d += 64) {
            out.w[d] = n_sub > 0 ? sub.w[d] : 0;
            out.n[d] = n_sub > 0 ? sub.n[d] : 0;
        }
        for (int j = lane; j < n_k; j += 64) {
            const bool own = j % world == rank;
            const int js = j / world;
            if (out.obj_by_k) out.obj_by_k[int64_t(f) * n_k + j] = own ? sub.obj_by_k[int64_t(f) * n_sub + js] : kInf;
            if (out.status) out.status[int64_t(f) * n_k + j] = own ? sub.status[int64_t(f) * n_sub + js] : INT32_MIN;
        }
    } else if (mode == 1) {  // after MIN(obj_value): the k this rank offers for the global minimum
        if (lane == 0) {
            const int bk = n_sub > 0 ? sub.best_k[f] : 0;
            out.best_k[f] = bk > 0 && sub.obj_value[f] == out.obj_value[f] ? bk : INT32_MAX;
        }
    } else {  // after MIN(k): only the owner keeps its (w, n) for the SUM
        const int bk = n_sub > 0 ? sub.best_k[f] : 0;
        const int kmin = out.best_k[f];
        if (bk != kmin || kmin == INT32_MAX)
            for (int64_t d = d0 + lane; d < d1; d += 64) out.w[d] = out.n[d] = 0;
    }
}

__global__ __launch_bounds__(256) void halda_shard_final_kernel(int nf, halda_fleet_result out) {
    const int f = blockIdx.x * 256 + threadIdx.x;
    if (f < nf && out.best_k[f] == INT32_MAX) out.best_k[f] = 0;  // no rank has a feasible k
}

int nccl_fail(ncclResult_t r, const char *what) {
    return fail(HALDA_E_HIP, std::string(what) + ": " + ncclGetErrorString(r));
}
#define NCCL_TRY(expr)                                     \
    do {                                                   \
        ncclResult_t r_ = (expr);                          \
        if (r_ != ncclSuccess) return nccl_fail(r_, #expr); \
    } while (0)

}  // namespace

extern "C" {

int halda_version(void) { return HALDA_ABI_VERSION; }

int halda_last_error(char *buf, size_t len) {
    if (buf && len) std::snprintf(buf, len, "%s", g_err.c_str());
    return int(g_err.size());
}

int64_t halda_lds_bytes(int32_t max_cols, int32_t max_R1, int32_t max_tab, int32_t max_tab_kc) {
    if (max_R1 < 1 || max_R1 > kMaxR1) return -1;
    const int mmax = (max_cols - 1) / 7 + 1;
    const int64_t tab = std::max<int64_t>(1, max_tab > 0 ? int64_t(max_tab) + mmax : 0);
    const int64_t tab_kc = max_tab_kc > 0 ? int64_t(max_tab_kc) + mmax : 0;
    return std::max(slice_bytes_for(mmax, max_R1, int(tab), 0), slice_bytes_for(mmax, max_R1, 0, int(tab_kc)));
}

int halda_init(int device_ordinal, void **ctx_out) {
    if (!ctx_out) return fail(HALDA_E_ARG, "ctx is NULL");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
        return fail(HALDA_E_NODEV, "no HIP device visible (libhalda needs an MI355X / gfx950)");
    if (device_ordinal < 0 || device_ordinal >= count)
        return fail(HALDA_E_NODEV, "device ordinal " + std::to_string(device_ordinal) + " out of range");
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device_ordinal));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(HALDA_E_NODEV, std::string("libhalda is built for gfx950, device is ") + prop.gcnArchName);
    HIP_TRY(hipSetDevice(device_ordinal));
    Ctx *c = new Ctx();
    c->device = device_ordinal;
    c->cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    if (hipMalloc(&c->hb_flag, 256) != hipSuccess || hipMemset(c->hb_flag, 0, 256) != hipSuccess) {
        delete c;
        return fail(HALDA_E_HIP, "hand-back flag allocation failed");
    }
    const char *tp = std::getenv("HALDA_TWO_PASS");
    c->two_pass = !(tp && tp[0] == '0');
    const char *fp = std::getenv("HALDA_FLEETS_PATH");
    c->fleets_fused = !(fp && std::strcmp(fp, "csr") == 0);
    c->seg_sweep = !(fp && std::strcmp(fp, "wave") == 0);
    const char *sw = std::getenv("HALDA_SWEEP_WAVES");
    c->sweep_waves = sw ? std::atoi(sw) : 0;
    const char *xs = std::getenv("HALDA_XCD_SWIZZLE");
    c->xcd_swizzle = !(xs && xs[0] == '0');
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipEventCreate(&c->evs) != hipSuccess || hipEventCreate(&c->evk) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_order, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_host, hipEventDisableTiming) != hipSuccess ||
        hipEventCreate(&c->evf0) != hipSuccess || hipEventCreate(&c->evf1) != hipSuccess ||
        hipEventCreate(&c->evfm) != hipSuccess) {
        halda_free(c);
        return fail(HALDA_E_HIP, "stream/event creation failed");
    }
    *ctx_out = c;
    return HALDA_OK;
}

void halda_free(void *ctx) {
    Ctx *c = static_cast<Ctx *>(ctx);
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->scratch) (void)hipFree(c->scratch);
    if (c->pinned) (void)hipHostFree(c->pinned);
    if (c->work) (void)hipFree(c->work);
    if (c->hb_flag) (void)hipFree(c->hb_flag);
    if (c->fleet_scratch) (void)hipFree(c->fleet_scratch);
    if (c->gtab) (void)hipFree(c->gtab);
    if (c->fflag) (void)hipFree(c->fflag);
    if (c->shard) (void)hipFree(c->shard);
    if (c->ev_order) (void)hipEventDestroy(c->ev_order);
    if (c->ev_host) (void)hipEventDestroy(c->ev_host);
    if (c->evf0) (void)hipEventDestroy(c->evf0);
    if (c->evf1) (void)hipEventDestroy(c->evf1);
    if (c->evfm) (void)hipEventDestroy(c->evfm);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->evs) (void)hipEventDestroy(c->evs);
    if (c->evk) (void)hipEventDestroy(c->evk);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int halda_solve_batch_device(void *ctx, const halda_batch *in, halda_result *out, void *stream) {
    Ctx *c = static_cast<Ctx *>(ctx);
    if (!c || !in || !out) return fail(HALDA_E_ARG, "NULL ctx/in/out");
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->stream;
    return launch(c, *in, *out, s);
}

int halda_last_kernel_ms(void *ctx, double *ms) {
    Ctx *c = static_cast<Ctx *>(ctx);
    if (!c || !ms) return fail(HALDA_E_ARG, "NULL ctx/ms");
    if (!c->timed) return fail(HALDA_E_ARG, "no solve has been launched on this context");
    HIP_TRY(hipEventSynchronize(c->ev1));
    float f = 0.f;
    HIP_TRY(hipEventElapsedTime(&f, c->ev0, c->ev1));
    *ms = f;
    return HALDA_OK;
}

int halda_last_solve_kernel_ms(void *ctx, double *ms) {
    Ctx *c = static_cast<Ctx *>(ctx);
    if (!c || !ms) return fail(HALDA_E_ARG, "NULL ctx/ms");
    if (!c->timed) return fail(HALDA_E_ARG, "no solve has been launched on this context");
    HIP_TRY(hipEventSynchronize(c->ev1));
    float f = 0.f;
    HIP_TRY(hipEventElapsedTime(&f, c->evs, c->ev1));
    *ms = f;
    return HALDA_OK;
}

int halda_set_timing(void *ctx, int on) {
    Ctx *c = static_cast<Ctx *>(ctx);
    if (!c) return fail(HALDA_E_ARG, "NULL ctx");
    c->timing = on != 0;
    if (!c->timing) c->timed = false;
    return HALDA_OK;
}

int halda_last_phase_ms(void *ctx, double *ms3) {
    Ctx *c = static_cast<Ctx *>(ctx);
    if (!c || !ms3) return fail(HALDA_E_ARG, "NULL ctx/ms");
    if (!c->timed) return fail(HALDA_E_ARG, "no solve has been launched on this context");
    HIP_TRY(hipEventSynchronize(c->ev1));
    float a = 0.f, b = 0.f, d = 0.f;
    HIP_TRY(hipEventElapsedTime(&a, c->ev0, c->evk));
    HIP_TRY(hipEventElapsedTime(&b, c->evk, c->evs));
    HIP_TRY(hipEventElapsedTime(&d, c->evs, c->ev1));
    ms3[0] = a;
    ms3[1] = b;
    ms3[2] = d;
    return HALDA_OK;
}

int halda_set_fleets_path(void *ctx, int path) {
    Ctx *c = static_cast<Ctx *>(ctx);
    if (!c) return fail(HALDA_E_ARG, "NULL ctx");
    if (path < 0 || path > 4)
        return fail(HALDA_E_ARG, "path must be 0 (CSR), 1 (fused), 2 (fused, one fleet per wave), 3 (fused, k = 1 "
                                 "by DP) or 4 (fused, segment kernel instead of the k-slot kernel)");
    c->fleets_fused = path != 0;
    c->seg_sweep = path == 1 || path == 4;
    c->kslot_sweep = path == 1;
    c->k1_force_dp = path == 3;
    return HALDA_OK;
}

int halda_last_fleet_ms(void *ctx, double *ms8) {
    Ctx *c = static_cast<Ctx *>(ctx);
    if (!c || !ms8) return fail(HALDA_E_ARG, "NULL ctx/ms");
    if (!c->fleet_timed) return fail(HALDA_E_ARG, "no timed halda_solve_fleets call on this context");
    HIP_TRY(hipEventSynchronize(c->evf1));
    for (int i = 0; i < 9; ++i) ms8[i] = 0.0;
    if (c->last_fleet_fused) {
        float a = 0.f, b = 0.f;
        if (c->fleet_two) {
            HIP_TRY(hipEventElapsedTime(&a, c->evf0, c->evfm));
            HIP_TRY(hipEventElapsedTime(&b, c->evfm, c->evf1));
            ms8[c->fleet_kslot ? 8 : c->fleet_seg ? 7 : 0] = a;
            ms8[1] = b;
        } else {
            HIP_TRY(hipEventElapsedTime(&a, c->evf0, c->evf1));
            ms8[c->fleet_reg_alone ? 0 : 1] = a;  // the register launch or the table launch alone
        }
        return HALDA_OK;
    }
    if (!c->timed) return fail(HALDA_E_ARG, "no timed launch on this context");
    float lo = 0.f, a = 0.f, b = 0.f, d = 0.f, pk = 0.f;
    HIP_TRY(hipEventElapsedTime(&lo, c->evf0, c->ev0));
    HIP_TRY(hipEventElapsedTime(&a, c->ev0, c->evk));
    HIP_TRY(hipEventElapsedTime(&b, c->evk, c->evs));
    HIP_TRY(hipEventElapsedTime(&d, c->evs, c->ev1));
    HIP_TRY(hipEventElapsedTime(&pk, c->ev1, c->evf1));
    ms8[2] = lo;
    ms8[3] = a;
    ms8[4] = b;
    ms8[5] = d;
    ms8[6] = pk;
    return HALDA_OK;
}

#ifdef HALDA_STAMPS
int halda_debug_stamps(unsigned long long *out, int n_inst) {
    const int n = std::min(n_inst, kStampInst);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_halda_stamps), sizeof(unsigned long long) * kStamps * n));
    return n;
}
#endif

int halda_solve_fleets(void *ctx, const halda_model *model, const halda_fleets *fleets, const int32_t *ks,
                       int32_t n_k, halda_fleet_result *out, void *stream) {
    Ctx *c = static_cast<Ctx *>(ctx);
    if (!c || !model || !fleets || !ks || !out) return fail(HALDA_E_ARG, "NULL ctx/model/fleets/ks/out");
    const halda_fleets &F = *fleets;
    if (F.n_fleets <= 0) return HALDA_OK;
    if (n_k <= 0 || n_k > 1024) return fail(HALDA_E_ARG, "n_k must be in 1..1024");
    if (F.min_devices < 1 || F.max_devices < F.min_devices || F.max_devices > 4096)
        return fail(HALDA_E_ARG, "halda_fleets: need 1 <= min_devices <= max_devices <= 4096");
    if (!F.dev_off || !F.os_class || !F.flags || !F.scpu_b1 || !F.sgpu_b1 || !F.T_cpu || !F.T_gpu ||
        !F.t_kvcpy_cpu || !F.t_kvcpy_gpu || !F.t_ram2vram || !F.t_vram2ram || !F.t_comm || !F.s_disk ||
        !F.d_avail_ram || !F.c_cpu || !F.c_gpu || !F.d_avail_cuda || !F.d_avail_metal || !F.swap)
        return fail(HALDA_E_ARG, "halda_fleets has a NULL array");
    if (!out->best_k || !out->obj_value || !out->w || !out->n) return fail(HALDA_E_ARG, "halda_fleet_result: NULL");
    if (model->L < 1) return fail(HALDA_E_ARG, "model.L < 1");
    // ks (host memory): ascending, unique, positive; staged into the scratch below
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->stream;
    const int32_t *kh = ks;
    for (int j = 0; j < n_k; ++j)
        if (kh[j] < 1 || (j && kh[j] <= kh[j - 1])) return fail(HALDA_E_ARG, "ks must be ascending, unique, > 0");
    if (c->fleets_fused && n_k <= 64) return sweep_fleets(c, *model, F, ks, n_k, *out, s);  // orders itself
    {
        const int rc = order_after_previous(c, s);  // fleet_scratch / last_lowered are per context
        if (rc != HALDA_OK) return rc;
    }
    const LowerDims D = lower_dims(F.max_devices, n_k);
    const int64_t n_inst = int64_t(F.n_fleets) * n_k;
    if (n_inst > (int64_t(1) << 30) || int64_t(F.n_fleets) * D.nnz > (int64_t(1) << 31) - 1)
        return fail(HALDA_E_ARG, "batch too large for one call");
    // scratch layout
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off += (bytes + 255) & ~size_t(255); return o; };
    const size_t o_ncols = take(4 * n_inst), o_nrows = take(4 * n_inst), o_csr = take(8 * n_inst),
                 o_col = take(8 * n_inst), o_row = take(8 * n_inst),
                 o_rp = take(4 * size_t(F.n_fleets) * size_t(D.rows + 1)), o_ci = take(4 * size_t(F.n_fleets) * D.nnz),
                 o_val = take(8 * size_t(F.n_fleets) * D.nnz), o_c = take(8 * n_inst * D.cols),
                 o_clb = take(8 * n_inst * D.cols), o_cub = take(8 * n_inst * D.cols),
                 o_rlb = take(8 * n_inst * D.rows), o_rub = take(8 * n_inst * D.rows), o_int = take(n_inst * D.cols),
                 o_offs = take(24 * size_t(F.n_fleets)), o_st = take(4 * n_inst), o_x = take(8 * n_inst * D.cols),
                 o_obj = take(8 * n_inst), o_db = take(8 * n_inst), o_gap = take(8 * n_inst), o_nodes = take(8 * n_inst),
                 o_ks = take(4 * size_t(n_k));
    if (off > c->fleet_scratch_bytes) {
        if (c->fleet_scratch) HIP_TRY(hipFree(c->fleet_scratch));
        c->fleet_scratch = nullptr;
        c->fleet_scratch_bytes = 0;
        HIP_TRY(hipMalloc(&c->fleet_scratch, off));
        c->fleet_scratch_bytes = off;
    }
    char *base = static_cast<char *>(c->fleet_scratch);
    // the k list travels with the stream (pageable source: the copy is staged before the call returns)
    int32_t *ks_dev = reinterpret_cast<int32_t *>(base + o_ks);
    HIP_TRY(hipMemcpyAsync(ks_dev, ks, sizeof(int32_t) * size_t(n_k), hipMemcpyHostToDevice, s));
    LowerOut O;
    O.n_cols = reinterpret_cast<int32_t *>(base + o_ncols);
    O.n_rows = reinterpret_cast<int32_t *>(base + o_nrows);
    O.csr_off = reinterpret_cast<int64_t *>(base + o_csr);
    O.col_off = reinterpret_cast<int64_t *>(base + o_col);
    O.row_off = reinterpret_cast<int64_t *>(base + o_row);
    O.row_ptr = reinterpret_cast<int32_t *>(base + o_rp);
    O.col_idx = reinterpret_cast<int32_t *>(base + o_ci);
    O.val = reinterpret_cast<double *>(base + o_val);
    O.c = reinterpret_cast<double *>(base + o_c);
    O.col_lb = reinterpret_cast<double *>(base + o_clb);
    O.col_ub = reinterpret_cast<double *>(base + o_cub);
    O.row_lb = reinterpret_cast<double *>(base + o_rlb);
    O.row_ub = reinterpret_cast<double *>(base + o_rub);
    O.integrality = reinterpret_cast<uint8_t *>(base + o_int);
    O.offs = reinterpret_cast<double *>(base + o_offs);
    c->fleet_timed = false;
    c->last_fleet_fused = false;
    if (c->timing) HIP_TRY(hipEventRecord(c->evf0, s));
    hipLaunchKernelGGL(halda_lower_kernel, dim3(unsigned(F.n_fleets)), dim3(64), 0, s, *model, F, ks_dev, int(n_k), D,
                       O);
    HIP_TRY(hipGetLastError());
    // the lowered batch and its shape summary (R = W - M with lb(w) = 1 on every device)
    halda_batch b = {};
    b.n_inst = int32_t(n_inst);
    b.max_cols = int32_t(D.cols);
    int64_t r1_k1 = 0, r1_kc = 0;
    for (int j = 0; j < n_k; ++j) {
        const int64_t r1 = int64_t(model->L / kh[j]) - F.min_devices + 1;
        if (kh[j] == 1) r1_k1 = std::max(r1_k1, r1);
        else r1_kc = std::max(r1_kc, r1);
    }
    const int64_t r1max = std::max<int64_t>(1, std::max(r1_k1, r1_kc));
    const int64_t tk1 = r1_k1 > 0 ? int64_t(F.max_devices) * r1_k1 : 0, tkc = r1_kc > 0 ? int64_t(F.max_devices) * r1_kc : 0;
    if (r1max > kMaxR1 || tk1 > (1 << 27) || tkc > (1 << 27))
        return fail(HALDA_E_ARG, "fleet shape out of range: (L / k_min - min_devices + 1) * max_devices > 2^27");
    b.max_R1 = int32_t(r1max);
    b.max_tab = int32_t(tk1);
    b.max_tab_kc = int32_t(tkc);
    b.n_cols = O.n_cols;
    b.n_rows = O.n_rows;
    b.csr_off = O.csr_off;
    b.col_off = O.col_off;
    b.row_off = O.row_off;
    b.row_ptr = O.row_ptr;
    b.col_idx = O.col_idx;
    b.val = O.val;
    b.c = O.c;
    b.col_lb = O.col_lb;
    b.col_ub = O.col_ub;
    b.row_lb = O.row_lb;
    b.row_ub = O.row_ub;
    b.integrality = O.integrality;
    b.mip_rel_gap = 0.0;
    b.mip_abs_gap = 0.0;
    b.time_limit = 0.0;
    halda_result r;
    r.status = reinterpret_cast<int32_t *>(base + o_st);
    r.x = reinterpret_cast<double *>(base + o_x);
    r.obj_lin = reinterpret_cast<double *>(base + o_obj);
    r.dual_bound = reinterpret_cast<double *>(base + o_db);
    r.gap = reinterpret_cast<double *>(base + o_gap);
    r.nodes = reinterpret_cast<int64_t *>(base + o_nodes);
    const int rc = launch(c, b, r, s);
    if (rc != HALDA_OK) return rc;
    hipLaunchKernelGGL(halda_pick_kernel, dim3(unsigned(F.n_fleets)), dim3(64), 0, s, b, r, F, int(n_k),
                       static_cast<const double *>(O.offs), *out, D.cols);
    HIP_TRY(hipGetLastError());
    if (c->timing) {
        HIP_TRY(hipEventRecord(c->evf1, s));
        c->fleet_timed = true;
    }
    c->last_lowered = b;
    c->last_solved = r;
    c->have_lowered = true;
    return HALDA_OK;
}

// Synchronous halda_solve_fleets on HOST arrays: copies the table in, solves, copies results out.
constexpr size_t kZeroCopyBytes = size_t(1) << 20;

int halda_solve_fleets_host(void *ctx, const halda_model *model, const halda_fleets *fh, const int32_t *ks,
                            int32_t n_k, halda_fleet_result *out_h) {
    Ctx *c = static_cast<Ctx *>(ctx);
    if (!c || !model || !fh || !ks || !out_h) return fail(HALDA_E_ARG, "NULL ctx/model/fleets/ks/out");
    if (fh->n_fleets <= 0) return HALDA_OK;
    if (!fh->dev_off) return fail(HALDA_E_ARG, "halda_fleets.dev_off is NULL");
    const int64_t nf = fh->n_fleets, nd = fh->dev_off[nf];
    if (nd < nf || n_k <= 0) return fail(HALDA_E_ARG, "bad device count / n_k");
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off += (bytes + 255) & ~size_t(255); return o; };
    const size_t o_doff = take(8 * (nf + 1)), o_cls = take(nd), o_fl = take(nd), o_f64 = take(8 * nd * 10),
                 o_i64 = take(8 * nd * 6);
    const bool xsel = out_h->x_off && (out_h->x || out_h->c);
    const size_t o_xoff = xsel ? take(8 * size_t(nf) * n_k) : 0;
    const size_t o_bk = take(4 * nf), o_obj = take(8 * nf), o_w = take(4 * nd),
                 o_n = take(4 * nd), o_obk = take(8 * nf * n_k), o_st = take(4 * nf * n_k);
    // x / c extent: the dense layout, or the caller's compact one (x_off, host memory)
    size_t xs = size_t(nf) * n_k * (7 * size_t(std::max(fh->max_devices, 1)) + 1);
    if (xsel) {
        int64_t ext = 0;
        for (int64_t f = 0; f < nf; ++f) {
            const int64_t N = 7 * (fh->dev_off[f + 1] - fh->dev_off[f]) + 1;
            for (int j = 0; j < n_k; ++j) {
                const int64_t a = out_h->x_off[f * n_k + j];
                if (a >= 0) ext = std::max(ext, a + N);
            }
        }
        xs = size_t(ext);
    }
    const size_t o_x = out_h->x ? take(8 * xs) : 0, o_c = out_h->c ? take(8 * xs) : 0;
    if (off > c->scratch_bytes) {
        if (c->scratch) HIP_TRY(hipFree(c->scratch));
        c->scratch = nullptr;
        c->scratch_bytes = 0;
        HIP_TRY(hipMalloc(&c->scratch, off));
        c->scratch_bytes = off;
    }
    char *base = static_cast<char *>(c->scratch);
    // inputs are packed into pinned host memory and cross PCIe in ONE copy (results likewise)
    if (off > c->pinned_bytes) {
        if (c->pinned) HIP_TRY(hipHostFree(c->pinned));
        c->pinned = nullptr;
        c->pinned_bytes = 0;
        HIP_TRY(hipHostMalloc(&c->pinned, off, hipHostMallocDefault));
        c->pinned_bytes = off;
    }
    char *pin = static_cast<char *>(c->pinned);
    auto up = [&](size_t o, const void *src, size_t bytes) {
        std::memcpy(pin + o, src, bytes);
        return hipSuccess;
    };
    halda_fleets d = *fh;
    HIP_TRY(up(o_doff, fh->dev_off, 8 * (nf + 1)));
    HIP_TRY(up(o_cls, fh->os_class, nd));
    HIP_TRY(up(o_fl, fh->flags, nd));
    const double *f64[10] = {fh->scpu_b1, fh->sgpu_b1, fh->T_cpu, fh->T_gpu, fh->t_kvcpy_cpu,
                             fh->t_kvcpy_gpu, fh->t_ram2vram, fh->t_vram2ram, fh->t_comm, fh->s_disk};
    const int64_t *i64[6] = {fh->d_avail_ram, fh->c_cpu, fh->c_gpu, fh->d_avail_cuda, fh->d_avail_metal, fh->swap};
    for (int a = 0; a < 10; ++a) {
        if (!f64[a] || !fh->os_class || !fh->flags) return fail(HALDA_E_ARG, "halda_fleets has a NULL array");
        HIP_TRY(up(o_f64 + 8 * nd * a, f64[a], 8 * nd));
    }
    for (int a = 0; a < 6; ++a) {
        if (!i64[a]) return fail(HALDA_E_ARG, "halda_fleets has a NULL array");
        HIP_TRY(up(o_i64 + 8 * nd * a, i64[a], 8 * nd));
    }
    // small calls (a single halda_solve: ~8 KB in, ~70 KB out) skip both copies: the kernels read the
    // table from and write the results to the pinned buffer itself, across PCIe, and the host polls
    // the completion event instead of sleeping in a stream synchronisation
    if (xsel) HIP_TRY(up(o_xoff, out_h->x_off, 8 * size_t(nf) * n_k));
    const bool zc = off <= kZeroCopyBytes;
    if (zc) {
        void *dp = nullptr;
        HIP_TRY(hipHostGetDevicePointer(&dp, c->pinned, 0));
        base = static_cast<char *>(dp);
    } else {
        HIP_TRY(hipMemcpyAsync(base, pin, o_bk, hipMemcpyHostToDevice, s));  // the table (and x_off)
    }
    auto F64 = [&](int a) { return reinterpret_cast<const double *>(base + o_f64 + 8 * nd * a); };
    auto I64 = [&](int a) { return reinterpret_cast<const int64_t *>(base + o_i64 + 8 * nd * a); };
    d.dev_off = reinterpret_cast<const int64_t *>(base + o_doff);
    d.os_class = reinterpret_cast<const uint8_t *>(base + o_cls);
    d.flags = reinterpret_cast<const uint8_t *>(base + o_fl);
    d.scpu_b1 = F64(0); d.sgpu_b1 = F64(1); d.T_cpu = F64(2); d.T_gpu = F64(3); d.t_kvcpy_cpu = F64(4);
    d.t_kvcpy_gpu = F64(5); d.t_ram2vram = F64(6); d.t_vram2ram = F64(7); d.t_comm = F64(8); d.s_disk = F64(9);
    d.d_avail_ram = I64(0); d.c_cpu = I64(1); d.c_gpu = I64(2); d.d_avail_cuda = I64(3); d.d_avail_metal = I64(4);
    d.swap = I64(5);
    halda_fleet_result r;
    r.best_k = reinterpret_cast<int32_t *>(base + o_bk);
    r.obj_value = reinterpret_cast<double *>(base + o_obj);
    r.w = reinterpret_cast<int32_t *>(base + o_w);
    r.n = reinterpret_cast<int32_t *>(base + o_n);
    r.obj_by_k = reinterpret_cast<double *>(base + o_obk);
    r.status = reinterpret_cast<int32_t *>(base + o_st);
    r.x = out_h->x ? reinterpret_cast<double *>(base + o_x) : nullptr;
    r.c = out_h->c ? reinterpret_cast<double *>(base + o_c) : nullptr;
    r.x_off = xsel ? reinterpret_cast<const int64_t *>(base + o_xoff) : nullptr;
    // zero-copy through the fused sweep: the kernels skip the zero x / c of non-optimal instances
    // (stores across PCIe, most of a one-fleet k-sweep's time); the copy-out below zero-fills them
    const bool host_zero = zc && c->fleets_fused && (r.x || r.c) && !xsel;
    c->x_zero = !host_zero;
    const int rc = halda_solve_fleets(ctx, model, &d, ks, n_k, &r, s);
    c->x_zero = true;
    if (rc != HALDA_OK) return rc;
    if (zc) {
        HIP_TRY(hipEventRecord(c->ev_host, s));
        hipError_t q;
        while ((q = hipEventQuery(c->ev_host)) == hipErrorNotReady) {
        }
        HIP_TRY(q);
    } else {
        HIP_TRY(hipMemcpyAsync(pin + o_bk, base + o_bk, off - o_bk, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    auto down = [&](void *dst, size_t o, size_t bytes) {
        if (dst) std::memcpy(dst, pin + o, bytes);
        return hipSuccess;
    };
    HIP_TRY(down(out_h->best_k, o_bk, 4 * nf));
    HIP_TRY(down(out_h->obj_value, o_obj, 8 * nf));
    HIP_TRY(down(out_h->w, o_w, 4 * nd));
    HIP_TRY(down(out_h->n, o_n, 4 * nd));
    HIP_TRY(down(out_h->obj_by_k, o_obk, 8 * nf * n_k));
    HIP_TRY(down(out_h->status, o_st, 4 * nf * n_k));
    if (host_zero) {
        // per (fleet, k): the kernel's x / c where the instance is optimal, zeros elsewhere
        const size_t per = xs / (size_t(nf) * n_k);
        const int32_t *st = reinterpret_cast<const int32_t *>(pin + o_st);
        for (size_t i = 0; i < size_t(nf) * n_k; ++i) {
            const bool opt = st[i] == HALDA_STATUS_OPTIMAL;
            for (int a = 0; a < 2; ++a) {
                double *dst = a == 0 ? out_h->x : out_h->c;
                if (!dst) continue;
                if (opt) std::memcpy(dst + i * per, pin + (a == 0 ? o_x : o_c) + 8 * i * per, 8 * per);
                else std::memset(dst + i * per, 0, 8 * per);
            }
        }
    } else {
        HIP_TRY(down(out_h->x, o_x, 8 * xs));
        HIP_TRY(down(out_h->c, o_c, 8 * xs));
    }
    return HALDA_OK;
}

// ---------------------------------------------------------------- several GPUs, one process
// The fleets of one call are independent: a multi-device context deals them out in contiguous
// blocks, one host thread per device runs halda_solve_fleets_host on its block, and the results
// land in the caller's arrays at the block's offsets. No collective is needed (the argmin over k is
// per fleet, on the device that solved it); multi-process / multi-node callers use one halda_init
// context per rank and torch.distributed / RCCL around it (distilp_amd/distributed.py).
struct MultiCtx {
    std::vector<void *> ctxs;
};

int halda_init_multi(int n_dev, const int *ordinals, void **mctx) {
    if (!mctx || n_dev < 1 || n_dev > 64 || !ordinals) return fail(HALDA_E_ARG, "halda_init_multi: bad arguments");
    MultiCtx *m = new MultiCtx();
    for (int i = 0; i < n_dev; ++i) {
        void *c = nullptr;
        const int rc = halda_init(ordinals[i], &c);
        if (rc != HALDA_OK) {
            for (void *o : m->ctxs) halda_free(o);
            delete m;
            return rc;
        }
        m->ctxs.push_back(c);
    }
    *mctx = m;
    return HALDA_OK;
}

void halda_free_multi(void *mctx) {
    MultiCtx *m = static_cast<MultiCtx *>(mctx);
    if (!m) return;
    for (void *c : m->ctxs) halda_free(c);
    delete m;
}

int halda_solve_fleets_multi(void *mctx, const halda_model *model, const halda_fleets *fh, const int32_t *ks,
                             int32_t n_k, halda_fleet_result *out_h) {
    MultiCtx *m = static_cast<MultiCtx *>(mctx);
    if (!m || !model || !fh || !ks || !out_h || !fh->dev_off) return fail(HALDA_E_ARG, "NULL argument");
    const int nd = int(m->ctxs.size()), nf = fh->n_fleets;
    if (nf <= 0) return HALDA_OK;
    const int64_t xs = 7 * int64_t(std::max(fh->max_devices, 1)) + 1;
    std::vector<std::vector<int64_t>> offs(nd), xoffs(nd);
    std::vector<int> rcs(nd, HALDA_OK);
    std::vector<std::string> errs(nd);
    std::vector<std::thread> th;
    for (int r = 0; r < nd; ++r) {
        const int base = nf / nd, extra = nf % nd;
        const int lo = r * base + std::min(r, extra), hi = lo + base + (r < extra ? 1 : 0);
        if (hi <= lo) continue;
        const int64_t d0 = fh->dev_off[lo];
        offs[r].resize(size_t(hi - lo + 1));
        for (int f = lo; f <= hi; ++f) offs[r][size_t(f - lo)] = fh->dev_off[f] - d0;
        th.emplace_back([&, r, lo, hi, d0]() {
            halda_fleets sub = *fh;  // min / max devices stay the call's (valid bounds for the block)
            sub.n_fleets = hi - lo;
            sub.dev_off = offs[r].data();
            sub.os_class = fh->os_class + d0;
            sub.flags = fh->flags + d0;
            sub.scpu_b1 = fh->scpu_b1 + d0; sub.sgpu_b1 = fh->sgpu_b1 + d0; sub.T_cpu = fh->T_cpu + d0;
            sub.T_gpu = fh->T_gpu + d0; sub.t_kvcpy_cpu = fh->t_kvcpy_cpu + d0; sub.t_kvcpy_gpu = fh->t_kvcpy_gpu + d0;
            sub.t_ram2vram = fh->t_ram2vram + d0; sub.t_vram2ram = fh->t_vram2ram + d0; sub.t_comm = fh->t_comm + d0;
            sub.s_disk = fh->s_disk + d0; sub.d_avail_ram = fh->d_avail_ram + d0; sub.c_cpu = fh->c_cpu + d0;
            sub.c_gpu = fh->c_gpu + d0; sub.d_avail_cuda = fh->d_avail_cuda + d0;
            sub.d_avail_metal = fh->d_avail_metal + d0; sub.swap = fh->swap + d0;
            halda_fleet_result o = *out_h;
            o.best_k = out_h->best_k + lo;
            o.obj_value = out_h->obj_value + lo;
            o.w = out_h->w + d0;
            o.n = out_h->n + d0;
            o.obj_by_k = out_h->obj_by_k ? out_h->obj_by_k + int64_t(lo) * n_k : nullptr;
            o.status = out_h->status ? out_h->status + int64_t(lo) * n_k : nullptr;
            if (out_h->x_off) {  // compact layout: the block's offsets relative to its first slot
                int64_t b0 = INT64_MAX;
                for (int64_t i = int64_t(lo) * n_k; i < int64_t(hi) * n_k; ++i)
                    if (out_h->x_off[i] >= 0) b0 = std::min(b0, out_h->x_off[i]);
                if (b0 == INT64_MAX) b0 = 0;
                xoffs[r].resize(size_t(hi - lo) * size_t(n_k));
                for (int64_t i = int64_t(lo) * n_k; i < int64_t(hi) * n_k; ++i)
                    xoffs[r][size_t(i - int64_t(lo) * n_k)] = out_h->x_off[i] >= 0 ? out_h->x_off[i] - b0 : -1;
                o.x_off = xoffs[r].data();
                o.x = out_h->x ? out_h->x + b0 : nullptr;
                o.c = out_h->c ? out_h->c + b0 : nullptr;
            } else {
                o.x = out_h->x ? out_h->x + int64_t(lo) * n_k * xs : nullptr;
                o.c = out_h->c ? out_h->c + int64_t(lo) * n_k * xs : nullptr;
            }
            rcs[r] = halda_solve_fleets_host(m->ctxs[size_t(r)], model, &sub, ks, n_k, &o);
            if (rcs[r] != HALDA_OK) errs[r] = g_err;
        });
    }
    for (auto &t : th) t.join();
    for (int r = 0; r < nd; ++r)
        if (rcs[r] != HALDA_OK) return fail(rcs[r], "device " + std::to_string(r) + ": " + errs[r]);
    return HALDA_OK;
}

int halda_comm_unique_id(void *id128) {
    if (!id128) return fail(HALDA_E_ARG, "NULL id");
    ncclUniqueId id;
    NCCL_TRY(ncclGetUniqueId(&id));
    std::memcpy(id128, &id, sizeof(id));
    return HALDA_OK;
}

int halda_comm_init(void **comm, int world, int rank, const void *id128, int device_ordinal) {
    if (!comm || !id128 || world < 1 || rank < 0 || rank >= world) return fail(HALDA_E_ARG, "halda_comm_init: bad arguments");
    HIP_TRY(hipSetDevice(device_ordinal));
    ncclUniqueId id;
    std::memcpy(&id, id128, sizeof(id));
    ncclComm_t c = nullptr;
    NCCL_TRY(ncclCommInitRank(&c, world, id, rank));
    *comm = c;
    return HALDA_OK;
}

void halda_comm_destroy(void *comm) {
    if (comm) (void)ncclCommDestroy(static_cast<ncclComm_t>(comm));
}

int halda_solve_fleets_sharded(void *ctx, void *comm, const halda_model *model, const halda_fleets *fleets,
                               const int32_t *ks, int32_t n_k, halda_fleet_result *out, void *stream) {
    Ctx *c = static_cast<Ctx *>(ctx);
    if (!c || !comm || !model || !fleets || !ks || !out) return fail(HALDA_E_ARG, "NULL argument");
    if (out->x || out->c) return fail(HALDA_E_ARG, "halda_solve_fleets_sharded: x / c are not gathered (pass NULL)");
    if (!out->best_k || !out->obj_value || !out->w || !out->n) return fail(HALDA_E_ARG, "halda_fleet_result: NULL");
    ncclComm_t cm = static_cast<ncclComm_t>(comm);
    int world = 0, rank = 0;
    NCCL_TRY(ncclCommCount(cm, &world));
    NCCL_TRY(ncclCommUserRank(cm, &rank));
    const halda_fleets &F = *fleets;
    const int64_t nf = F.n_fleets;
    if (nf <= 0) return HALDA_OK;
    if (n_k <= 0 || n_k > 1024) return fail(HALDA_E_ARG, "n_k must be in 1..1024");
    for (int j = 0; j < n_k; ++j)
        if (ks[j] < 1 || (j && ks[j] <= ks[j - 1])) return fail(HALDA_E_ARG, "ks must be ascending, unique, > 0");
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->stream;
    // this rank's k's: ks[rank], ks[rank + world], ... (halda_solve_distributed deals them the same way)
    std::vector<int32_t> mine;
    for (int j = rank; j < n_k; j += world) mine.push_back(ks[j]);
    const int n_sub = int(mine.size());
    // device count: nf * M for one fleet size, else read back from dev_off[nf] (a synchronous copy)
    int64_t nd = nf * F.max_devices;
    if (F.min_devices != F.max_devices) {
        HIP_TRY(hipMemcpyAsync(&nd, F.dev_off + nf, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off += (bytes + 255) & ~size_t(255); return o; };
    const size_t o_bk = take(4 * nf), o_obj = take(8 * nf), o_w = take(4 * size_t(nd)), o_n = take(4 * size_t(nd)),
                 o_obk = take(8 * nf * std::max(n_sub, 1)), o_st = take(4 * nf * std::max(n_sub, 1));
    if (off > c->shard_bytes) {
        if (c->shard) HIP_TRY(hipFree(c->shard));
        c->shard = nullptr;
        c->shard_bytes = 0;
        HIP_TRY(hipMalloc(&c->shard, off));
        c->shard_bytes = off;
    }
    char *base = static_cast<char *>(c->shard);
    halda_fleet_result sub = {};
    sub.best_k = reinterpret_cast<int32_t *>(base + o_bk);
    sub.obj_value = reinterpret_cast<double *>(base + o_obj);
    sub.w = reinterpret_cast<int32_t *>(base + o_w);
    sub.n = reinterpret_cast<int32_t *>(base + o_n);
    sub.obj_by_k = out->obj_by_k ? reinterpret_cast<double *>(base + o_obk) : nullptr;
    sub.status = out->status ? reinterpret_cast<int32_t *>(base + o_st) : nullptr;
    {
        const int rc = order_after_previous(c, s);  // the shard scratch is per context
        if (rc != HALDA_OK) return rc;
    }
    if (n_sub > 0) {
        const int rc = halda_solve_fleets(ctx, model, fleets, mine.data(), n_sub, &sub, s);
        if (rc != HALDA_OK) return rc;
    }
    const halda_fleet_result o = *out;
    hipLaunchKernelGGL(halda_shard_kernel, dim3(unsigned(nf)), dim3(64), 0, s, 0, int(n_k), n_sub, rank, world,
                       F.dev_off, sub, o);
    HIP_TRY(hipGetLastError());
    NCCL_TRY(ncclAllReduce(o.obj_value, o.obj_value, size_t(nf), ncclFloat64, ncclMin, cm, s));
    hipLaunchKernelGGL(halda_shard_kernel, dim3(unsigned(nf)), dim3(64), 0, s, 1, int(n_k), n_sub, rank, world,
                       F.dev_off, sub, o);
    HIP_TRY(hipGetLastError());
    NCCL_TRY(ncclAllReduce(o.best_k, o.best_k, size_t(nf), ncclInt32, ncclMin, cm, s));
    hipLaunchKernelGGL(halda_shard_kernel, dim3(unsigned(nf)), dim3(64), 0, s, 2, int(n_k), n_sub, rank, world,
                       F.dev_off, sub, o);
    HIP_TRY(hipGetLastError());
    NCCL_TRY(ncclGroupStart());
    NCCL_TRY(ncclAllReduce(o.w, o.w, size_t(nd), ncclInt32, ncclSum, cm, s));
    NCCL_TRY(ncclAllReduce(o.n, o.n, size_t(nd), ncclInt32, ncclSum, cm, s));
    if (o.obj_by_k) NCCL_TRY(ncclAllReduce(o.obj_by_k, o.obj_by_k, size_t(nf) * n_k, ncclFloat64, ncclMin, cm, s));
    if (o.status) NCCL_TRY(ncclAllReduce(o.status, o.status, size_t(nf) * n_k, ncclInt32, ncclMax, cm, s));
    NCCL_TRY(ncclGroupEnd());
    hipLaunchKernelGGL(halda_shard_final_kernel, dim3(unsigned((nf + 255) / 256)), dim3(256), 0, s, int(nf), o);
    HIP_TRY(hipGetLastError());
    return HALDA_OK;
}

int halda_last_lowered(void *ctx, halda_batch *lowered, halda_result *solved) {
    Ctx *c = static_cast<Ctx *>(ctx);
    if (!c || !lowered || !solved) return fail(HALDA_E_ARG, "NULL ctx/lowered/solved");
    if (!c->have_lowered)
        return fail(HALDA_E_ARG, "no lowered batch: the last halda_solve_fleets call ran the fused sweep "
                                 "(halda_set_fleets_path(ctx, 0) selects the CSR pipeline)");
    *lowered = c->last_lowered;
    *solved = c->last_solved;
    return HALDA_OK;
}

int halda_solve_batch(void *ctx, const halda_batch *in_h, halda_result *out_h) {
    Ctx *c = static_cast<Ctx *>(ctx);
    if (!c || !in_h || !out_h) return fail(HALDA_E_ARG, "NULL ctx/in/out");
    const halda_batch &h = *in_h;
    const int n = h.n_inst;
    if (n < 0) return fail(HALDA_E_ARG, "n_inst < 0");
    if (n == 0) return HALDA_OK;
    if (!h.n_cols || !h.n_rows || !h.csr_off || !h.col_off || !h.row_off || !h.row_ptr || !h.col_idx || !h.val ||
        !h.c || !h.col_lb || !h.col_ub || !h.row_lb || !h.row_ub || !h.integrality)
        return fail(HALDA_E_ARG, "halda_batch has a NULL array");
    if (!out_h->status || !out_h->x || !out_h->obj_lin || !out_h->dual_bound || !out_h->gap || !out_h->nodes)
        return fail(HALDA_E_ARG, "halda_result has a NULL array");
    int64_t n_colsum = 0, n_rowsum = 0, n_rp = 0, nnz = 0;
    halda_batch d = h;
    const bool need_summary = h.max_cols == 0 && h.max_R1 == 0 && h.max_tab == 0 && h.max_tab_kc == 0;
    if (need_summary) d.max_R1 = 1;
    for (int i = 0; i < n; ++i) {
        const int N = h.n_cols[i], m = h.n_rows[i];
        if (N < 1 || m < 1 || h.csr_off[i] < 0 || h.col_off[i] < 0 || h.row_off[i] < 0)
            return fail(HALDA_E_ARG, "instance " + std::to_string(i) + ": bad sizes/offsets");
        n_colsum = std::max<int64_t>(n_colsum, h.col_off[i] + N);
        n_rowsum = std::max<int64_t>(n_rowsum, h.row_off[i] + m);
        n_rp = std::max<int64_t>(n_rp, h.csr_off[i] + m + 1);
        nnz = std::max<int64_t>(nnz, int64_t(h.row_ptr[h.csr_off[i] + m]));
        if (need_summary) {
            d.max_cols = std::max(d.max_cols, N);
            if ((N - 1) % 7 == 0) {
                const int M = (N - 1) / 7;
                const double W = h.row_ub[h.row_off[i] + m - 1];
                double sum = 0.0;
                for (int j = 0; j < M; ++j) sum += std::ceil(h.col_lb[h.col_off[i] + j]);
                const double Rr = W - sum;
                if (Rr >= 0 && Rr < 1e6) {
                    const int R1 = int(Rr) + 1;
                    d.max_R1 = std::max(d.max_R1, R1);
                    if (h.c[h.col_off[i] + 7 * M] > 0) d.max_tab_kc = std::max(d.max_tab_kc, M * R1);
                    else d.max_tab = std::max(d.max_tab, M * R1);
                }
            }
        }
    }
    HIP_TRY(hipSetDevice(c->device));
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off += (bytes + 255) & ~size_t(255); return o; };
    const size_t o_ncols = take(4 * n), o_nrows = take(4 * n), o_csr = take(8 * n), o_col = take(8 * n),
                 o_row = take(8 * n), o_rp = take(4 * n_rp), o_ci = take(4 * nnz), o_val = take(8 * nnz),
                 o_c = take(8 * n_colsum), o_clb = take(8 * n_colsum), o_cub = take(8 * n_colsum),
                 o_rlb = take(8 * n_rowsum), o_rub = take(8 * n_rowsum), o_int = take(n_colsum),
                 o_st = take(4 * n), o_x = take(8 * n_colsum), o_obj = take(8 * n), o_db = take(8 * n),
                 o_gap = take(8 * n), o_nodes = take(8 * n);
    if (off > c->scratch_bytes) {
        if (c->scratch) HIP_TRY(hipFree(c->scratch));
        c->scratch = nullptr;
        c->scratch_bytes = 0;
        HIP_TRY(hipMalloc(&c->scratch, off));
        c->scratch_bytes = off;
    }
    char *base = static_cast<char *>(c->scratch);
    hipStream_t s = c->stream;
    {
        const int rc = order_after_previous(c, s);
        if (rc != HALDA_OK) return rc;
    }
    auto up = [&](size_t o, const void *src, size_t bytes) {
        return hipMemcpyAsync(base + o, src, bytes, hipMemcpyHostToDevice, s);
    };
    HIP_TRY(up(o_ncols, h.n_cols, 4 * n));
    HIP_TRY(up(o_nrows, h.n_rows, 4 * n));
    HIP_TRY(up(o_csr, h.csr_off, 8 * n));
    HIP_TRY(up(o_col, h.col_off, 8 * n));
    HIP_TRY(up(o_row, h.row_off, 8 * n));
    HIP_TRY(up(o_rp, h.row_ptr, 4 * n_rp));
    HIP_TRY(up(o_ci, h.col_idx, 4 * nnz));
    HIP_TRY(up(o_val, h.val, 8 * nnz));
    HIP_TRY(up(o_c, h.c, 8 * n_colsum));
    HIP_TRY(up(o_clb, h.col_lb, 8 * n_colsum));
    HIP_TRY(up(o_cub, h.col_ub, 8 * n_colsum));
    HIP_TRY(up(o_rlb, h.row_lb, 8 * n_rowsum));
    HIP_TRY(up(o_rub, h.row_ub, 8 * n_rowsum));
    HIP_TRY(up(o_int, h.integrality, n_colsum));
    HIP_TRY(hipMemsetAsync(base + o_x, 0, 8 * n_colsum, s));
    d.n_cols = reinterpret_cast<const int32_t *>(base + o_ncols);
    d.n_rows = reinterpret_cast<const int32_t *>(base + o_nrows);
    d.csr_off = reinterpret_cast<const int64_t *>(base + o_csr);
    d.col_off = reinterpret_cast<const int64_t *>(base + o_col);
    d.row_off = reinterpret_cast<const int64_t *>(base + o_row);
    d.row_ptr = reinterpret_cast<const int32_t *>(base + o_rp);
    d.col_idx = reinterpret_cast<const int32_t *>(base + o_ci);
    d.val = reinterpret_cast<const double *>(base + o_val);
    d.c = reinterpret_cast<const double *>(base + o_c);
    d.col_lb = reinterpret_cast<const double *>(base + o_clb);
    d.col_ub = reinterpret_cast<const double *>(base + o_cub);
    d.row_lb = reinterpret_cast<const double *>(base + o_rlb);
    d.row_ub = reinterpret_cast<const double *>(base + o_rub);
    d.integrality = reinterpret_cast<const uint8_t *>(base + o_int);
    d.x0 = d.y0 = nullptr;
    halda_result r;
    r.status = reinterpret_cast<int32_t *>(base + o_st);
    r.x = reinterpret_cast<double *>(base + o_x);
    r.obj_lin = reinterpret_cast<double *>(base + o_obj);
    r.dual_bound = reinterpret_cast<double *>(base + o_db);
    r.gap = reinterpret_cast<double *>(base + o_gap);
    r.nodes = reinterpret_cast<int64_t *>(base + o_nodes);
    int rc = launch(c, d, r, s);
    if (rc != HALDA_OK) return rc;
    auto down = [&](void *dst, size_t o, size_t bytes) {
        return hipMemcpyAsync(dst, base + o, bytes, hipMemcpyDeviceToHost, s);
    };
    HIP_TRY(down(out_h->status, o_st, 4 * n));
    HIP_TRY(down(out_h->x, o_x, 8 * n_colsum));
    HIP_TRY(down(out_h->obj_lin, o_obj, 8 * n));
    HIP_TRY(down(out_h->dual_bound, o_db, 8 * n));
    HIP_TRY(down(out_h->gap, o_gap, 8 * n));
    HIP_TRY(down(out_h->nodes, o_nodes, 8 * n));
    HIP_TRY(hipStreamSynchronize(s));
    return HALDA_OK;
}

}  // extern "C"
