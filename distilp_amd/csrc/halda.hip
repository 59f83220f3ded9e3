// libhalda — exact batched solver for fixed-k HALDA MILPs on MI355X (gfx950).
//
// Replaces the per-(fleet, k) call scipy.optimize.milp -> HiGHS made by the
// reference at src/distilp/solver/halda_p_solver.py:340-346; the C ABI is in
// include/halda.h, the design (and why the DP is exact) in DESIGN.md.
//
// One 256-thread workgroup (4 wave64s) solves one instance, entirely on chip:
//   1. validate + decode the CSR MILP into per-device records in LDS (every
//      thread owns rows / devices; the CSR, bounds and costs are read once,
//      coalesced, from HBM);
//   2. table phase: for every device i and every extra-layer count
//      e = w_i - lb(w_i) in [0, R], R = W - sum_i lb(w_i), find the best GPU
//      split n (the cost is convex piecewise-linear in n, so only the interval
//      ends and the slack kinks are evaluated) -> G[i][e] (cost), H[i][e]
//      (least cycle time, only when k > 1);
//   3. wave 0 runs a min-plus DP over sum(e) (state width R + 1, which is the
//      slack of the problem, 17 at M=64/W=80), and for k > 1 a pruned
//      ascending scan over cycle-time thresholds T (min (k-1)T + S(T));
//   4. backtrack, then all threads rebuild x (w, n, slacks, stalls z, cycle C).
// All floating-point arithmetic keeps the reference's operation order
// (compiled with -ffp-contract=off).

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

#include "halda.h"

namespace {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
constexpr int kRows = 4;             // capacity rows per device (link, RAM/Metal cap, <= 2 VRAM)
constexpr int kMaxRowNnz = 8;        // widest HALDA row (cycle rows: 6 device cols + z + C)
constexpr double kSlackEps = 1e-9;   // a capacity row counts as met within 1e-9 layers (oracle: same)
constexpr double kInf = __builtin_huge_val();

// per-device double fields (SoA, index f * Mmax + i)
enum { DD_CW, DD_CN, DD_CS0, DD_CS1, DD_CS2, DD_CS3, DD_R1W, DD_R2W, DD_RHS1, DD_RHS2, DD_G, DD_H, kDevD };
// per-device int fields
enum {
    DI_WLO, DI_WHI, DI_NLO, DI_NHI, DI_SLO0, DI_SLO1, DI_SLO2, DI_SLO3,
    DI_SHI0, DI_SHI1, DI_SHI2, DI_SHI3, DI_NROW, DI_HAVE1, DI_HAVE2, DI_WSOL, kDevI
};
// block scalars (ints)
enum { SC_FLAGS, SC_SUMWLO, SC_NODES, SC_STATUS, kScI = 8 };
// flag bits
enum { F_UNSUPPORTED = 1, F_INFEASIBLE = 2, F_TOO_LARGE = 4 };

struct Layout {
    int64_t dd, di, rows, tab, choice, dp, red, sci, total;
};

__host__ __device__ inline int64_t align16(int64_t x) { return (x + 15) & ~int64_t(15); }

__host__ __device__ inline Layout make_layout(int mmax, int r1max, int tab, int tab_kc) {
    Layout L;
    int64_t o = 0;
    L.dd = o;     o = align16(o + int64_t(mmax) * kDevD * 8);
    L.di = o;     o = align16(o + int64_t(mmax) * kDevI * 4);
    L.rows = o;   o = align16(o + int64_t(mmax) * kRows * 16);
    int64_t tb = int64_t(tab) * 8 > int64_t(tab_kc) * 16 ? int64_t(tab) * 8 : int64_t(tab_kc) * 16;
    L.tab = o;    o = align16(o + tb);
    L.choice = o; o = align16(o + (tab > tab_kc ? tab : tab_kc));
    L.dp = o;     o = align16(o + 2 * int64_t(r1max) * 8);
    L.red = o;    o = align16(o + 8 * kWaves * 2);
    L.sci = o;    o = align16(o + 4 * kScI);
    L.total = o;
    return L;
}

struct Lds {
    double *dd;
    int *di;
    int *rows;
    double *G, *H;
    uint8_t *choice;
    double *D0, *D1;
    double *red;
    int *sc;
    int mmax;
    __device__ double &d(int f, int i) const { return dd[f * mmax + i]; }
    __device__ int &n(int f, int i) const { return di[f * mmax + i]; }
    __device__ int *row(int i, int q) const { return rows + (i * kRows + q) * 4; }
};

__device__ inline void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ inline double wave_min(double v) {
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
    return v;
}
__device__ inline double wave_max(double v) {
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
}

// Least slacks (s1, s2, s3, t) for integer (w, n); false when a row cannot be met.
// Row (kind, u, v, K): slack rows need s_kind >= u*w + v*n + K with
// K = ceil(-rhs/beta - eps); pure (w, n) rows need u*w + v*n <= K.
__device__ inline bool least_slacks(const Lds &L, int i, int w, int n, int s[4]) {
    s[0] = L.n(DI_SLO0, i); s[1] = L.n(DI_SLO1, i); s[2] = L.n(DI_SLO2, i); s[3] = L.n(DI_SLO3, i);
    const int nr = L.n(DI_NROW, i);
    for (int q = 0; q < nr; ++q) {
        const int *r = L.row(i, q);
        const int val = r[1] * w + r[2] * n;
        if (r[0] < 0) {
            if (val > r[3]) return false;
        } else {
            const int need = val + r[3];
            if (need > s[r[0]]) s[r[0]] = need;
        }
    }
    return s[0] <= L.n(DI_SHI0, i) && s[1] <= L.n(DI_SHI1, i) && s[2] <= L.n(DI_SHI2, i) &&
           s[3] <= L.n(DI_SHI3, i);
}

// Objective contribution of device i (same term order as c.x in the reference).
__device__ inline double dev_cost(const Lds &L, int i, int w, int n, const int s[4]) {
    double g = L.d(DD_CW, i) * double(w);
    g = g + L.d(DD_CN, i) * double(n);
    g = g + L.d(DD_CS0, i) * double(s[0]);
    g = g + L.d(DD_CS1, i) * double(s[1]);
    g = g + L.d(DD_CS2, i) * double(s[2]);
    g = g + L.d(DD_CS3, i) * double(s[3]);
    return g;
}

// Cycle rows: C >= P + z, C >= Q - z with z >= 0  ->  least C = max(P, (P+Q)/2).
__device__ inline void dev_cycle(const Lds &L, int i, int w, int n, const int s[4], double &P, double &Q) {
    double a1 = L.d(DD_R1W, i) * double(w), a2 = L.d(DD_R2W, i) * double(w);
    const double tail[5] = {L.d(DD_CN, i) * double(n), L.d(DD_CS0, i) * double(s[0]), L.d(DD_CS1, i) * double(s[1]),
                            L.d(DD_CS2, i) * double(s[2]), L.d(DD_CS3, i) * double(s[3])};
#pragma unroll
    for (int b = 0; b < 5; ++b) {
        a1 = a1 + tail[b];
        a2 = a2 + tail[b];
    }
    P = a1 - L.d(DD_RHS1, i);
    Q = a2 - L.d(DD_RHS2, i);
}

// Best GPU split n for device i holding w layers. The cost is convex
// piecewise-linear in integer n (every slack is max(lb, affine in n with slope
// -1/0/+1) and has a non-negative price), so its minimum over the feasible
// interval sits at an interval end or a kink. Ties -> smallest n.
__device__ inline bool best_split(const Lds &L, int i, int w, double &g_out, int &n_out, int s_out[4]) {
    int nL = L.n(DI_NLO, i), nU = L.n(DI_NHI, i);
    int cand[2 + kRows + 12];
    int nc = 0;
    const int nr = L.n(DI_NROW, i);
    for (int q = 0; q < nr; ++q) {
        const int *r = L.row(i, q);
        const int kind = r[0], u = r[1], v = r[2], K = r[3];
        if (v == 0) continue;
        if (kind < 0) {  // u w + v n <= K
            if (v > 0) nU = min(nU, K - u * w); else nL = max(nL, u * w - K);
        } else {
            const int slo = L.n(DI_SLO0 + kind, i), shi = L.n(DI_SHI0 + kind, i);
            if (v > 0) nU = min(nU, shi - K - u * w); else nL = max(nL, u * w + K - shi);
            cand[nc++] = v * (slo - K - u * w);  // where the slack starts to bind
            for (int q2 = 0; q2 < q; ++q2) {     // two rows pricing the same slack with opposite slopes
                const int *r2 = L.row(i, q2);
                if (r2[0] == kind && r2[2] == -v) {
                    const int num = (r2[1] * w + r2[3]) - (u * w + K);  // (v - v2) n = num, v - v2 = +-2
                    const int nn = v > 0 ? num : -num;
                    const int f = nn >= 0 ? nn / 2 : -((-nn + 1) / 2);
                    cand[nc++] = f;
                    cand[nc++] = f + 1;
                }
            }
        }
    }
    if (nL > nU) return false;
    double best = kInf;
    int bn = -1;
    int bs[4] = {0, 0, 0, 0};
    cand[nc++] = nL;
    cand[nc++] = nU;
    for (int k = 0; k < nc; ++k) {
        const int nn = min(max(cand[k], nL), nU);
        int s[4];
        if (!least_slacks(L, i, w, nn, s)) continue;
        const double g = dev_cost(L, i, w, nn, s);
        if (g < best || (g == best && nn < bn)) {
            best = g; bn = nn;
            bs[0] = s[0]; bs[1] = s[1]; bs[2] = s[2]; bs[3] = s[3];
        }
    }
    if (bn < 0) return false;
    g_out = best; n_out = bn;
    s_out[0] = bs[0]; s_out[1] = bs[1]; s_out[2] = bs[2]; s_out[3] = bs[3];
    return true;
}

// Min-plus DP over devices by ONE wave: D[r] = least sum of G over a prefix
// using r extra layers; choice[i][r] = e taken by device i. With use_T only
// entries whose cycle time H <= T are allowed. Returns D_M[R].
__device__ double wave_dp(const Lds &L, int M, int R, bool use_T, double T, int lane) {
    const int R1 = R + 1;
    double *D0 = L.D0, *D1 = L.D1;
    for (int r = lane; r < R1; r += 64) D0[r] = r == 0 ? 0.0 : kInf;
    wave_sync();
    for (int i = 0; i < M; ++i) {
        const double *Gi = L.G + i * R1;
        const double *Hi = L.H + i * R1;
        for (int r = lane; r < R1; r += 64) {
            double best = kInf;
            int be = 255;
            for (int e = 0; e <= r; ++e) {
                const double g = Gi[e];
                if (use_T && !(Hi[e] <= T)) continue;
                const double val = D0[r - e] + g;
                if (val < best) { best = val; be = e; }
            }
            D1[r] = best;
            L.choice[i * R1 + r] = uint8_t(be);
        }
        wave_sync();
        double *t = D0; D0 = D1; D1 = t;
    }
    return D0[R];
}

// lane 0: walk the choices back; wsol[i] = lb(w_i) + e_i
__device__ void backtrack(const Lds &L, int M, int R) {
    const int R1 = R + 1;
    int r = R;
    for (int i = M - 1; i >= 0; --i) {
        const int e = L.choice[i * R1 + r];
        L.n(DI_WSOL, i) = L.n(DI_WLO, i) + e;
        r -= e;
    }
}

__global__ __launch_bounds__(kBlock) void halda_solve_kernel(halda_batch B, halda_result Rz, int mmax, int r1max,
                                                               int tab, int tab_kc) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const Layout lay = make_layout(mmax, r1max, tab, tab_kc);
    Lds L;
    L.dd = reinterpret_cast<double *>(smem + lay.dd);
    L.di = reinterpret_cast<int *>(smem + lay.di);
    L.rows = reinterpret_cast<int *>(smem + lay.rows);
    L.G = reinterpret_cast<double *>(smem + lay.tab);
    L.choice = smem + lay.choice;
    L.D0 = reinterpret_cast<double *>(smem + lay.dp);
    L.D1 = L.D0 + r1max;
    L.red = reinterpret_cast<double *>(smem + lay.red);
    L.sc = reinterpret_cast<int *>(smem + lay.sci);
    L.mmax = mmax;

    const int inst = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int N = B.n_cols[inst], m = B.n_rows[inst];
    const int64_t co = B.col_off[inst], ro = B.row_off[inst];
    const int32_t *rp = B.row_ptr + B.csr_off[inst];

    auto finish = [&](int status) {
        if (tid == 0) {
            Rz.status[inst] = status;
            Rz.nodes[inst] = 0;
            Rz.obj_lin[inst] = kInf;
            Rz.dual_bound[inst] = status == HALDA_STATUS_INFEASIBLE ? kInf : -kInf;
            Rz.gap[inst] = kInf;
        }
    };
    if (N < 1 || (N - 1) % 7 != 0 || m < 1) { finish(HALDA_STATUS_UNSUPPORTED); return; }
    const int M = (N - 1) / 7, iC = 7 * M;
    if (M > mmax) { finish(HALDA_STATUS_TOO_LARGE); return; }

    if (tid < kScI) L.sc[tid] = 0;
    __syncthreads();

    // ---- equality row sum_i w_i = W and quick bound infeasibility
    const double Wd = B.row_ub[ro + m - 1];
    const int eqs = rp[m - 1], eqe = rp[m];
    if (!(B.row_lb[ro + m - 1] == Wd) || !(Wd >= 0.0 && Wd < 1e6 && Wd == floor(Wd)) || eqe - eqs != M) {
        finish(HALDA_STATUS_UNSUPPORTED);
        return;
    }
    const int W = int(Wd);
    for (int i = tid; i < M; i += kBlock) {
        if (B.col_idx[eqs + i] != i || B.val[eqs + i] != 1.0) atomicOr(&L.sc[SC_FLAGS], F_UNSUPPORTED);
        const double lb = B.col_lb[co + i], ub = B.col_ub[co + i];
        const int wlo = int(ceil(lb)), whi = int(floor(fmin(ub, Wd)));
        L.n(DI_WLO, i) = wlo;
        L.n(DI_WHI, i) = whi;
        atomicAdd(&L.sc[SC_SUMWLO], wlo);
        if (wlo > whi || lb < 0.0) atomicOr(&L.sc[SC_FLAGS], F_INFEASIBLE);
    }
    __syncthreads();
    {
        const int fl = L.sc[SC_FLAGS];
        if (fl & F_UNSUPPORTED) { finish(HALDA_STATUS_UNSUPPORTED); return; }
        if ((fl & F_INFEASIBLE) || L.sc[SC_SUMWLO] > W) { finish(HALDA_STATUS_INFEASIBLE); return; }
    }
    const int R = W - L.sc[SC_SUMWLO];
    const int R1 = R + 1;
    const double kc = B.c[co + iC];
    if (R1 > r1max || M * R1 > (kc > 0.0 ? tab_kc : tab)) { finish(HALDA_STATUS_TOO_LARGE); return; }
    L.H = L.G + M * R1;

    // ---- per-device costs and bounds
    for (int i = tid; i < M; i += kBlock) {
        int bad = 0;
        const double cw = B.c[co + i], cn = B.c[co + M + i];
        L.d(DD_CW, i) = cw;
        L.d(DD_CN, i) = cn;
        for (int b = 0; b < 6; ++b) bad |= B.integrality[co + b * M + i] != 1;
        bad |= B.integrality[co + 6 * M + i] != 0 || B.c[co + 6 * M + i] != 0.0;
        bad |= B.col_lb[co + 6 * M + i] != 0.0 || B.col_ub[co + 6 * M + i] != kInf;
        const double nlo = B.col_lb[co + M + i], nhi = B.col_ub[co + M + i];
        L.n(DI_NLO, i) = int(ceil(nlo));
        L.n(DI_NHI, i) = int(floor(fmin(nhi, Wd)));
        for (int s = 0; s < 4; ++s) {
            const double cs = B.c[co + (2 + s) * M + i];
            L.d(DD_CS0 + s, i) = cs;
            bad |= !(cs >= 0.0);
            L.n(DI_SLO0 + s, i) = int(ceil(B.col_lb[co + (2 + s) * M + i]));
            L.n(DI_SHI0 + s, i) = int(floor(fmin(B.col_ub[co + (2 + s) * M + i], 1e6)));
        }
        bad |= nlo < 0.0;
        L.n(DI_NROW, i) = 0;
        L.n(DI_HAVE1, i) = 0;
        L.n(DI_HAVE2, i) = 0;
        if (bad) atomicOr(&L.sc[SC_FLAGS], F_UNSUPPORTED);
    }
    if (tid == 0) {
        const bool ok = kc >= 0.0 && B.integrality[co + iC] == 0 && B.col_lb[co + iC] == 0.0 &&
                        B.col_ub[co + iC] == kInf;
        if (!ok) atomicOr(&L.sc[SC_FLAGS], F_UNSUPPORTED);
    }
    __syncthreads();

    // ---- rows: classify by nonzero pattern (one thread per row)
    for (int r = tid; r < m - 1; r += kBlock) {
        const int s = rp[r], e = rp[r + 1], nnz = e - s;
        const double rhs = B.row_ub[ro + r];
        int bad = B.row_lb[ro + r] != -kInf || nnz < 1 || nnz > kMaxRowNnz || !(fabs(rhs) < 1e300);
        int cols[kMaxRowNnz];
        double vals[kMaxRowNnz];
        for (int k = 0; k < kMaxRowNnz; ++k) {
            if (!bad && k < nnz) { cols[k] = B.col_idx[s + k]; vals[k] = B.val[s + k]; }
        }
        if (!bad && cols[nnz - 1] == iC) {
            // cycle row: busy(i) +- z_i - C <= rhs
            const int zc = nnz >= 2 ? cols[nnz - 2] : -1;
            const int dev = zc - 6 * M;
            bad |= vals[nnz - 1] != -1.0 || dev < 0 || dev >= M || fabs(vals[nnz - 2]) != 1.0;
            if (!bad) {
                const bool first = vals[nnz - 2] > 0.0;
                double coef[6] = {0, 0, 0, 0, 0, 0};
                for (int k = 0; k < nnz - 2; ++k) {
                    const int j = cols[k];
                    if (j >= 6 * M || j % M != dev) { bad = 1; break; }
                    coef[j / M] = vals[k];
                }
                // the non-w part of a cycle row must equal the device's objective terms
                bad |= coef[1] != L.d(DD_CN, dev);
                for (int b = 0; b < 4; ++b) bad |= coef[2 + b] != L.d(DD_CS0 + b, dev);
                if (!bad) {
                    if (first) {
                        L.d(DD_R1W, dev) = coef[0]; L.d(DD_RHS1, dev) = rhs;
                        atomicAdd(&L.n(DI_HAVE1, dev), 1);
                    } else {
                        L.d(DD_R2W, dev) = coef[0]; L.d(DD_RHS2, dev) = rhs;
                        atomicAdd(&L.n(DI_HAVE2, dev), 1);
                    }
                }
            }
        } else if (!bad) {
            // capacity / link row of one device: aw w + an n - beta s <= rhs
            int dev = -1, slack = -1;
            double aw = 0.0, an = 0.0, beta = 0.0;
            for (int k = 0; k < nnz; ++k) {
                const int j = cols[k], blk = j / M, i = j % M;
                if (j >= 6 * M || (dev >= 0 && i != dev)) { bad = 1; break; }
                dev = i;
                if (blk == 0) aw = vals[k];
                else if (blk == 1) an = vals[k];
                else if (slack >= 0) { bad = 1; break; }
                else { slack = blk - 2; beta = -vals[k]; }
            }
            int u = 0, v = 0, K = 0;
            if (!bad) {
                const double scale = slack >= 0 ? beta : fmax(fabs(aw), fabs(an));
                bad |= !(scale > 0.0);
                if (!bad) {
                    bad |= !(aw == 0.0 || fabs(aw) == scale) || !(an == 0.0 || fabs(an) == scale);
                    u = aw == 0.0 ? 0 : (aw > 0.0 ? 1 : -1);
                    v = an == 0.0 ? 0 : (an > 0.0 ? 1 : -1);
                    double kk;
                    if (slack >= 0) kk = ceil(-rhs / beta - kSlackEps);
                    else kk = floor((rhs + kSlackEps * fmax(1.0, fabs(rhs))) / scale);
                    bad |= !(fabs(kk) < 1e8);
                    K = int(kk);
                }
            }
            if (!bad) {
                const int q = atomicAdd(&L.n(DI_NROW, dev), 1);
                if (q >= kRows) bad = 1;
                else {
                    int *rw = L.row(dev, q);
                    rw[0] = slack; rw[1] = u; rw[2] = v; rw[3] = K;
                }
            }
        }
        if (bad) atomicOr(&L.sc[SC_FLAGS], F_UNSUPPORTED);
    }
    __syncthreads();
    for (int i = tid; i < M; i += kBlock)
        if (L.n(DI_HAVE1, i) != 1 || L.n(DI_HAVE2, i) != 1 || L.n(DI_NROW, i) > kRows)
            atomicOr(&L.sc[SC_FLAGS], F_UNSUPPORTED);
    __syncthreads();
    if (L.sc[SC_FLAGS] & F_UNSUPPORTED) { finish(HALDA_STATUS_UNSUPPORTED); return; }

    // ---- table phase: G[i][e], H[i][e] for w = lb(w_i) + e
    for (int p = tid; p < M * R1; p += kBlock) {
        const int i = p / R1, e = p - i * R1;
        const int w = L.n(DI_WLO, i) + e;
        double g = kInf, h = kInf;
        int n, s[4];
        if (w <= L.n(DI_WHI, i) && best_split(L, i, w, g, n, s)) {
            if (kc > 0.0) {
                double P, Q;
                dev_cycle(L, i, w, n, s, P, Q);
                h = fmax(0.0, Q >= P ? 0.5 * (P + Q) : P);
            }
        } else {
            g = kInf;
        }
        L.G[p] = g;
        if (kc > 0.0) L.H[p] = h;
    }
    __syncthreads();

    // ---- DP (wave 0); k > 1: ascending threshold scan with bound pruning
    if (wave == 0) {
        int nodes = 1;
        const double s_inf = wave_dp(L, M, R, false, 0.0, lane);
        int status = s_inf < kInf ? HALDA_STATUS_OPTIMAL : HALDA_STATUS_INFEASIBLE;
        if (status == HALDA_STATUS_OPTIMAL && kc > 0.0) {
            if (lane == 0) backtrack(L, M, R);
            wave_sync();
            double hmax = 0.0;
            for (int i = lane; i < M; i += 64) hmax = fmax(hmax, L.H[i * R1 + (L.n(DI_WSOL, i) - L.n(DI_WLO, i))]);
            hmax = wave_max(hmax);
            double best = kc * hmax + s_inf, bestT = kInf;
            // every assignment has max_i H_i >= T_lo = max_i min_e H[i][e]
            double tlo = 0.0;
            for (int i = lane; i < M; i += 64) {
                double mn = kInf;
                for (int e = 0; e < R1; ++e)
                    if (L.G[i * R1 + e] < kInf) mn = fmin(mn, L.H[i * R1 + e]);
                tlo = fmax(tlo, mn);
            }
            tlo = wave_max(tlo);
            double tprev = -1.0;
            while (true) {
                double t = kInf;
                for (int p = lane; p < M * R1; p += 64) {
                    const double h = L.H[p];
                    if (L.G[p] < kInf && h >= tlo && h > tprev) t = fmin(t, h);
                }
                t = wave_min(t);
                if (!(t < kInf) || kc * t + s_inf >= best) break;
                const double st = wave_dp(L, M, R, true, t, lane);
                ++nodes;
                if (st < kInf && kc * t + st < best) { best = kc * t + st; bestT = t; }
                tprev = t;
            }
            if (bestT < kInf) wave_dp(L, M, R, true, bestT, lane);
            else wave_dp(L, M, R, false, 0.0, lane);
            ++nodes;
        }
        if (lane == 0) {
            if (status == HALDA_STATUS_OPTIMAL) backtrack(L, M, R);
            L.sc[SC_STATUS] = status;
            L.sc[SC_NODES] = nodes;
        }
    }
    __syncthreads();
    if (L.sc[SC_STATUS] != HALDA_STATUS_OPTIMAL) {
        if (tid == 0) {
            Rz.status[inst] = L.sc[SC_STATUS];
            Rz.nodes[inst] = L.sc[SC_NODES];
            Rz.obj_lin[inst] = kInf;
            Rz.dual_bound[inst] = kInf;
            Rz.gap[inst] = kInf;
        }
        return;
    }

    // ---- rebuild x for the chosen w: n, least slacks, stall z, cycle time C
    for (int i = tid; i < M; i += kBlock) {
        const int w = L.n(DI_WSOL, i);
        double g = 0.0, P, Q;
        int n = 0, s[4] = {0, 0, 0, 0};
        best_split(L, i, w, g, n, s);
        dev_cycle(L, i, w, n, s, P, Q);
        double *x = Rz.x + co;
        x[i] = double(w);
        x[M + i] = double(n);
        x[2 * M + i] = double(s[0]);
        x[3 * M + i] = double(s[1]);
        x[4 * M + i] = double(s[2]);
        x[5 * M + i] = double(s[3]);
        x[6 * M + i] = Q > P ? 0.5 * (Q - P) : 0.0;
        L.d(DD_G, i) = g;
        L.d(DD_H, i) = Q >= P ? 0.5 * (P + Q) : P;
    }
    __syncthreads();
    if (wave == 0) {
        double h = 0.0;
        for (int i = lane; i < M; i += 64) h = fmax(h, L.d(DD_H, i));
        h = wave_max(h);
        if (lane == 0) {
            double obj = 0.0;
            for (int i = 0; i < M; ++i) obj = obj + L.d(DD_G, i);
            obj = obj + kc * h;
            Rz.x[co + iC] = h;
            Rz.status[inst] = HALDA_STATUS_OPTIMAL;
            Rz.obj_lin[inst] = obj;
            Rz.dual_bound[inst] = obj;
            Rz.gap[inst] = 0.0;
            Rz.nodes[inst] = L.sc[SC_NODES];
        }
    }
}

// ------------------------------------------------------------------ host side
thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                                   \
    do {                                                                                                \
        hipError_t e_ = (expr);                                                                         \
        if (e_ != hipSuccess) return fail(HALDA_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

struct Ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool timed = false;
    void *scratch = nullptr;
    size_t scratch_bytes = 0;
};

int64_t lds_for(int mmax, int r1max, int tab, int tab_kc) { return make_layout(mmax, r1max, tab, tab_kc).total; }

int launch(Ctx *ctx, const halda_batch &in, const halda_result &out, hipStream_t stream) {
    if (in.n_inst <= 0) return HALDA_OK;
    if (in.max_cols < 1 || in.max_R1 < 1 || in.max_tab < 0 || in.max_tab_kc < 0)
        return fail(HALDA_E_ARG, "halda_batch shape summary (max_cols/max_R1/max_tab/max_tab_kc) not set");
    const int mmax = (in.max_cols - 1) / 7 + 1;
    const int tab = in.max_tab > 0 ? in.max_tab : 1, tab_kc = in.max_tab_kc;
    const int64_t lds = lds_for(mmax, in.max_R1, tab, tab_kc);
    if (lds > 160 * 1024)
        return fail(HALDA_E_ARG, "batch needs " + std::to_string(lds) + " B of LDS per instance (> 160 KiB)");
    HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void *>(halda_solve_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
    HIP_TRY(hipEventRecord(ctx->ev0, stream));
    hipLaunchKernelGGL(halda_solve_kernel, dim3(in.n_inst), dim3(kBlock), size_t(lds), stream, in, out, mmax,
                       in.max_R1, tab, tab_kc);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(ctx->ev1, stream));
    ctx->timed = true;
    return HALDA_OK;
}

}  // namespace

extern "C" {

int halda_version(void) { return HALDA_ABI_VERSION; }

int halda_last_error(char *buf, size_t len) {
    if (buf && len) {
        std::snprintf(buf, len, "%s", g_err.c_str());
    }
    return int(g_err.size());
}

int64_t halda_lds_bytes(int32_t max_cols, int32_t max_R1, int32_t max_tab, int32_t max_tab_kc) {
    return lds_for((max_cols - 1) / 7 + 1, max_R1, max_tab > 0 ? max_tab : 1, max_tab_kc);
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
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
        delete c;
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
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
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
    // extents of the shared arrays
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
    // one grow-only device allocation, 256-B aligned sub-buffers
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
