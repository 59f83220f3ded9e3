// halda_solve.hpp -- the milp() replacement (halda_solve_batch): device records, the split / cycle-time
// primitives, the greedy exchange and the min-plus DP, the CSR decode, and the screen, k = 1 and
// general kernels.
// Part of libhalda's single translation unit: included by halda.hip inside its anonymous namespace
// (after halda_prims.hpp); not a standalone header.
#pragma once
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
                                    int mmax, int r1max, int tab, int tab_kc, ScreenOut &so,
                                    const uint8_t *settled, int *gen_flag, int launch_id, int nlim = kScreenPer) {
    // lane g < kScreenPer: header of instance i0 + g. Loads are branch-free (lanes
    // without an instance read a valid element and discard it) so that each round
    // trip's loads issue before the first wait. nlim < kScreenPer: only instances i0 .. i0 + nlim - 1
    // (the settled k = 1 kernel's screen of one instance, halda_solve_k1_settled_kernel).
    const int64_t my = i0 + lane;
    const bool own = lane < nlim && lane < kScreenPer && my < B.n_inst;
    const int64_t mc = own ? my : i0;
    const int N0 = B.n_cols[mc], m0 = B.n_rows[mc];
    const int64_t co0 = B.col_off[mc], ro0 = B.row_off[mc], cs0 = B.csr_off[mc];
    // a settled instance (the caller's proof of bound infeasibility, halda_solve_batch_device_settled) is
    // INFEASIBLE as it stands: none of its rows or bounds is read (only its header)
    const bool hint = own && settled && settled[mc] != 0;
    const int N = own ? N0 : 1, m = own ? m0 : 1;
    const int64_t co = own ? co0 : 0, ro = own ? ro0 : 0, cs = own ? cs0 : 0;
    int status = hint ? HALDA_STATUS_INFEASIBLE : 0;  // 0 = still open
    if (!status && (N < 1 || (N - 1) % 7 != 0 || m < 1)) status = HALDA_STATUS_UNSUPPORTED;
    const int M = status ? 0 : (N - 1) / 7;
    if (!status && M > mmax) status = HALDA_STATUS_TOO_LARGE;
    // round trip 2: equality-row extent and bounds, c[C] (lane g). Lanes without an unsettled instance
    // read the lines of the first lane that has one; a wave of settled instances alone reads nothing.
    const bool rd = own && !hint;
    const uint64_t rdm = __ballot(rd);
    const int src = rdm ? __builtin_ctzll(rdm) : 0;
    const int m_r = __shfl(m0, src), M_r = __shfl(M, src);
    const int64_t cs_r = shfl64(cs0, src), ro_r = shfl64(ro0, src), co_r = shfl64(co0, src);
    const int ma = max(rd ? m0 : m_r, 1);
    const int32_t *rp = B.row_ptr + (rd ? cs0 : cs_r);
    const int64_t rr = (rd ? ro0 : ro_r) + ma - 1;
    const int64_t ci = (rd ? co0 : co_r) + 7 * int64_t(max(rd ? M : M_r, 0));
    int eqs0 = 0, eqe0 = 0;
    double Wd0 = 0.0, Wl0 = 0.0, cC0 = 0.0;
    if (rdm) {
        eqs0 = rp[ma - 1];
        eqe0 = rp[ma];
        Wd0 = B.row_ub[rr];
        Wl0 = B.row_lb[rr];
        cC0 = B.c[ci];
    }
    const bool live = own && !status;
    const int eqs = live ? eqs0 : 0, eqe = live ? eqe0 : 0;
    const double Wd = live ? Wd0 : 0.0, Wl = live ? Wl0 : 0.0, cC = live ? cC0 : 0.0;
    if (!status && (!(Wl == Wd) || !(Wd >= 0.0 && Wd < 1e6 && Wd == floor(Wd)) || eqe - eqs != M))
        status = HALDA_STATUS_UNSUPPORTED;

    // round trip 3, per instance g (lane = device): its equality row entries -- loaded once for a run of
    // instances sharing the row (the k-instances of one fleet share its CSR) -- and the first
    // pre = min(M, W + 1) w lower bounds. Each bound is >= 0 or makes the instance infeasible by itself
    // (lb < 0, and ceil(lb) > W, are infeasible; NaN counts 0), so when those first bounds already need
    // more than W layers the instance is infeasible whatever the others are (bound infeasibility, M > W
    // = L / k: 8 of the 9 C3 instances), and the others are read only when they do not.
    int cv[kScreenPer];
    double vv[kScreenPer];
    double lbv[kScreenPer];
    int pre_[kScreenPer];
    const uint64_t open = __ballot(lane < kScreenPer && own && !status && M > 0);
    const int safe = open ? __shfl(eqs0, __builtin_ctzll(open)) : 0;
    const int64_t safe_c = open ? shfl64(co0, __builtin_ctzll(open)) : 0;
    int e_prev = -1, m_prev = -1;
#pragma unroll
    for (int g = 0; g < kScreenPer; ++g) {
        if (g >= nlim) break;
        const int stg = __shfl(status, g), eg = __shfl(eqs0, g);
        const int Mg = __shfl(M, g);
        const int64_t cg = shfl64(co0, g);
        const int Wg = int(__shfl(Wd, g));
        const bool og = open && i0 + g < B.n_inst && stg == 0;  // wave-uniform
        const bool in = og && lane < Mg;
        const int pre = og ? min(Mg, Wg + 1) : 0;
        pre_[g] = pre;
        if (g > 0 && og && eg == e_prev && Mg == m_prev) {  // the same row as the previous open instance
            cv[g] = cv[g - 1];
            vv[g] = vv[g - 1];
        } else {
            const int idx = in ? eg + lane : safe;
            const int c0 = open ? B.col_idx[idx] : 0;
            const double v0 = open ? B.val[idx] : 1.0;
            cv[g] = in ? c0 : lane;
            vv[g] = in ? v0 : 1.0;
        }
        if (og) {
            e_prev = eg;
            m_prev = Mg;
        }
        const bool lin = og && lane < pre;
        const double l0 = open ? B.col_lb[lin ? cg + lane : safe_c] : 0.0;
        lbv[g] = lin ? l0 : 0.0;
    }
    int verdict = CLS_DONE, vstatus = status;  // lane g: outcome of instance g
#pragma unroll
    for (int g = 0; g < kScreenPer; ++g) {
        if (i0 + g >= B.n_inst || g >= nlim) break;
        const int stg = __shfl(status, g);
        if (stg) continue;
        const int Mg = __shfl(M, g), eg = __shfl(eqs, g), pre = pre_[g];
        const int64_t cg = shfl64(co, g);
        const double Wg = __shfl(Wd, g);
        int bad = 0, infeas = 0, sumlo = 0;
        auto lbone = [&](double lb) {
            const int wlo = int(ceil(lb));
            infeas |= wlo > int(Wg) || lb < 0.0;
            sumlo += wlo;
        };
        if (lane < Mg) bad |= cv[g] != lane || vv[g] != 1.0;
        for (int i = lane + 64; i < Mg; i += 64) bad |= B.col_idx[eg + i] != i || B.val[eg + i] != 1.0;
        if (lane < pre) lbone(lbv[g]);
        for (int i = lane + 64; i < pre; i += 64) lbone(B.col_lb[cg + i]);
        bad = wave_or(bad | (infeas << 1));
        sumlo = wave_sum(sumlo);
        if (!bad && sumlo <= int(Wg) && pre < Mg) {  // the first bounds prove nothing: the rest of them
            infeas = 0;
            int rest = 0;
            for (int i = pre + lane; i < Mg; i += 64) {
                const double lb = B.col_lb[cg + i];
                const int wlo = int(ceil(lb));
                infeas |= wlo > int(Wg) || lb < 0.0;
                rest += wlo;
            }
            bad = wave_or(infeas << 1);
            sumlo += wave_sum(rest);
        }
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
    // the k > 1 general launch of this batch has work (it is gated on this flag)
    if (__ballot(own && verdict == CLS_GEN) && lane == 0) *gen_flag = launch_id;
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

// The screen of ONE instance by one wave (the settled k = 1 kernel's slow path: shapes its fast path does not
// take); returns the verdict on every lane.
__device__ inline int screen_one(const halda_batch &B, const halda_result &Rz, uint8_t *cls, int64_t i, int lane,
                                       int mmax, int r1max, int tab, int tab_kc, int *gen_flag, int launch_id) {
    ScreenOut so;
    screen_group(B, Rz, cls, i, lane, mmax, r1max, tab, tab_kc, so, nullptr, gen_flag, launch_id, 1);
    return __shfl(so.verdict, 0);
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
__device__ inline bool split_second(const Dev &d, int w, double &g, int &n, int s[4]) { return split_full(d, w, g, n, s); }

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
//
// Split over two waves of a k-slot workgroup (16-lane segments only, sp.part != 0): the scan's length
// is the workgroup's critical path, and each event is a dependent chain of reductions, so the
// candidate range is cut at T_a (the value of rank 4/8 among the devices' H at cap(T0) + 2;
// tools/scan_model.py on dumped C2 tables: the longest scan per wave 47 -> 28 events at the median) and
// the two parts run at once. Part 1 (the slot's own wave) takes the openings T <= T_a; part 2 (a helper wave)
// starts from an optimal capped allocation at T_a (the greedy's) and takes the openings above it,
// pruning with its own bound. Under ties (repeated devices) that allocation need not be the one the
// one scan holds at T_a, and it does not have to be: an exchange keeps ANY optimal capped allocation
// optimal (its largest taken increment lam and the set of useful openings are the same for every
// optimal allocation), and T never decreases (above), so part 2 prices the same S(T) as the one scan
// from T_a on (tests/test_scan_split_model.py, tests/test_gpu_ties.py). Part 1 then takes part 2's
// allocation only when strictly better, so the earliest T wins ties as in the one scan.
constexpr int kMaxSplitParts = 2;
struct SplitArea {  // per segment, in LDS
    // part 1 -> the helpers, after its leaf scan and phase-0 greedy (the helpers repeat neither)
    double s_inf, best0;
    int lo_sum, capsum;
    int pub;             // 0: not yet, 1: published, 2: part 1 does not scan (the helpers skip)
    int verdict;         // the helper's leaf check of part 1's rows (optimistic part 1): 0 not yet, 1 ok, 2 not
    int16_t lo[16], hi[16];  // each device's finite leaf range (R + 1 < 2^15: a split slot's tables fit LDS)
    // the helpers -> part 1
    double alt_best[kMaxSplitParts - 1];  // part p's best objective (+inf: nothing beat its start)
    int flag[kMaxSplitParts - 1];         // set once part p's alt_e / alt_best are final
    int alt_e[kMaxSplitParts - 1][16];    // part p's allocation (one int per segment lane)
};
struct ScanSplit {
    int part = 0;     // 0: no split, 1: the slot's own wave, 2: the helper
    int n_parts = 0;  // 2 (split) or 0
    SplitArea *ar = nullptr;
    bool fetch = false;  // part 1: s_inf / best0 come from the helper's phase 0 (published in ar)
    bool opt = false;    // part 1 may take rows finite at both ends without checking them (dp_pass_lanes)
#ifdef HALDA_STAMPS
    unsigned long long *prof = nullptr;  // g_halda_scanprof of this wave (part 1 only)
#endif
    int cut8 = 4;  // the cut's rank, in eighths of the way up (both parts use the same)
};

// Rank of v among the 16 lanes of its DPP row (ties: the lower lane first).
template <int R>
__device__ inline int rank_step(double v, int sl) {
    const double u = ror16<R>(v);
    const int j = (sl + R) & 15;
    return (u < v || (u == v && j < sl)) ? 1 : 0;
}
template <int... R>
__device__ inline int rank16(double v, int sl, std::integer_sequence<int, R...>) {
    return (rank_step<R + 1>(v, sl) + ...);
}

// Largest cap in [cap, hi] with H[cap] <= T, H nondecreasing on the row's finite range (checked by the
// leaf scan): eight entries per LDS round trip (the entries <= T are a prefix of each chunk).
__device__ inline int advance_cap(const double *H, int cap, int hi, double T) {
    while (cap < hi) {
        double hv[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) hv[t] = H[min(cap + 1 + t, hi)];
        int adv = 0;
#pragma unroll
        for (int t = 0; t < 8; ++t) adv += (cap + 1 + t <= hi && hv[t] <= T) ? 1 : 0;
        cap += adv;
        if (adv < 8) break;
    }
    return cap;
}

template <class SG>
__device__ bool kc_scan_incremental(const WaveCtx &w, const Inst &I, const SG &sg, double s_inf_in, double best0_in,
                                    int64_t &nodes, const LeafInfo &li0, const ScanSplit sp = ScanSplit{}) {
    double s_inf = s_inf_in, best0 = best0_in;
    const int M = I.M, R1 = I.R1, RS = I.RS;
    const double kc = I.kc;
    const int lane = sg.sl;  // device index within the problem
    if (M > SG::S || M < 2 || !li0.convex || !li0.mono || li0.empty) return false;
    HALDA_KSTAMP(3);
#ifdef HALDA_STAMPS  // diagnostic build: cycles per step, summed over the events (tools/scan_prof.py)
    unsigned long long pa[12] = {}, tp = __builtin_amdgcn_s_memtime();
#define HALDA_SCANPROF(slot, ...)                                        \
    do {                                                                 \
        asm volatile("" ::__VA_ARGS__);                                  \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();      \
        pa[slot] += t_ - tp;                                             \
        tp = t_;                                                         \
    } while (0)
#else
#define HALDA_SCANPROF(slot, ...) do {} while (0)
#endif
    const bool act = lane < M;
    const double *G = w.G + int64_t(act ? lane : 0) * RS, *H = w.H + int64_t(act ? lane : 0) * RS;
    const int lo = act ? li0.my_lo : 0, hi = act ? li0.my_hi : -1;
    const int need_total = (R1 - 1) - li0.lo_sum;
    if (need_total < 0 || need_total > li0.cap) return false;
    // start at T0 = max_i H_i(lo_i): every device can sit at its first allowed e
    double T = sg.max_f64(act ? H[lo] : -kInf);
    int cap = act ? advance_cap(H, lo, hi, T) : lo;
    HALDA_SCANPROF(5, "v"(cap), "v"(T));
    const int part = sp.part;
    double t_stop = kInf;  // the part's upper cut (inclusive)
    if constexpr (SG::S == 16) {
        if (part) {
            const bool has = act && cap < hi;  // a device with an opening past T0
            const double v2 = has ? H[min(cap + 2, hi)] : kInf;
            const int n = sg.sum_i(has ? 1 : 0);
            const int r2 = rank16(v2, lane, std::make_integer_sequence<int, 15>{});
            // the cut (> T0; +inf: no opening at all)
            // (rank sp.cut8 / 8 of the way up, 4/8 by default: measured 3/8 .. 6/8 with five k-slot
            // workgroups per CU; 5/8 was best at four, when part 1 first left its leaf checks and phase 0
            // to other waves)
            const double ta = sg.min_f64(has && r2 == (n - 1) * sp.cut8 / 8 ? v2 : kInf);
            t_stop = part == 1 ? ta : kInf;
            if (part > 1) {
                T = ta;
                if (act) cap = advance_cap(H, cap, hi, T);
            }
        }
    }
    HALDA_SCANPROF(6, "v"(cap), "v"(T), "v"(t_stop));
    // optimal capped allocation at T0 (a helper: at its lower cut) (greedy: every cap filled from lo, then the smallest increments)
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
    HALDA_SCANPROF(7, "v"(e), "v"(need));
    double S = sg.sum_f64(act ? G[e] : 0.0);
    HALDA_KSTAMP(4);
    if constexpr (SG::S == 16) {
        if (sp.part == 1 && sp.fetch) {  // the helper's phase 0 (its s_inf and bound), needed from here on
            while (sg.any(__hip_atomic_load(&sp.ar->pub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0))
                __builtin_amdgcn_s_sleep(1);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            s_inf = sp.ar->s_inf;
            best0 = sp.ar->best0;
        }
    }
    double best = best0;
    int bestE = -1;
    int64_t events = 0;
    // Only "useful" cap openings change the optimum: device i must sit at its cap (e_i == cap_i; a
    // device below its cap already declined a unit no worse than its next) and the unit its next cap
    // opens must be needed (allocation incomplete) or beat the largest taken unit lam. lam only
    // decreases, so a device that is not useful now never becomes useful except the one that just
    // took a unit; the scan therefore jumps T straight to the next useful opening and costs one
    // reduction per exchange instead of one per candidate T.
    // That holds in exact arithmetic. In floating point a leaf that is linear over a stretch (equal
    // increments: the same device twice, a homogeneous cluster) has increments that differ by
    // rounding, so "gn < lam" may become true for a device only after lam was re-formed from its own
    // twin's equal unit -- an opening whose H lies below the T already reached. T therefore never
    // decreases: such an opening is taken at the current T (its H is <= T, so it is allowed there), and
    // the recorded kc T + S stays the cost of an allocation whose cycle times are all <= T. The
    // exchanges it allows change S by rounding only.
    // Per lane, in registers: the next two openings (cap + 1, cap + 2: H and the unit each opens) and the
    // last two taken units (at e, e - 1), so that an event moves its two lanes by register shifts; the
    // LDS reads that refill the shifted-out entry are issued during the event and first used at a later
    // one. Every value is the one the reads at the event would give (the same two-entry differences).
    double hn = act && cap < hi ? H[cap + 1] : kInf;           // H of this device's next cap
    double gn = act && cap < hi ? G[cap + 1] - G[cap] : kInf;  // the unit it opens (cap -> cap + 1)
    double hn2 = act && cap + 1 < hi ? H[cap + 2] : kInf;      // the same one cap further
    double gn2 = act && cap + 1 < hi ? G[cap + 2] - G[cap + 1] : kInf;
    double lt = act && e > lo ? G[e] - G[e - 1] : -kInf;       // its last taken unit
    double lt2 = act && e - 1 > lo ? G[e - 1] - G[e - 2] : -kInf;  // the one below it
    double lam = -kInf;
    int lj = -1;
    if (need == 0) {
        lam = sg.max_f64(lt);
        lj = sg.highest(lt == lam);
        if (kc * T + S < best) {
            // a helper's start only bounds its pruning: a lower part already priced this allocation
            best = kc * T + S;
            bestE = part > 1 ? -1 : e;
        }
    }
    HALDA_SCANPROF(8, "v"(S), "v"(lam), "v"(hn), "v"(gn), "v"(lt), "v"(best));
    while (true) {
        // useful: at its cap, with a next cap (else hn = gn = +inf), and needed or beating lam
        const double lamU = need > 0 ? kInf : lam;
        const bool useful = (e == cap) & (gn < lamU);  // (no short circuit: one select, no branch)
        const double cand = useful ? hn : kInf;
        const double Tn = sg.min_f64(cand);
        const double Te = vmax_f64(T, Tn);  // (+inf when no opening is left)
        if (!(Tn < kInf) || !(kc * Te + s_inf < best) || Te > t_stop) break;
        HALDA_SCANPROF(0, "v"(Te));
        const int li = sg.lowest(cand == Tn);
        ++events;
        const double d = sg.bcast(gn, li);
        HALDA_SCANPROF(1, "v"(d));
        const bool swap = need == 0;  // else: fill
        // li takes the unit its new cap opens; lj gives back its largest taken unit (li == lj only
        // through the convexity tolerance: then both, e unchanged)
        const bool is_li = lane == li, is_lj = swap && lane == lj;
        const int cap_n = is_li ? cap + 1 : cap;
        const int e_n = is_li ? (is_lj ? e : e + 1) : (is_lj ? e - 1 : e);
        const double lt_n = is_li ? (is_lj ? lt : gn) : (is_lj ? lt2 : lt);
        double lt2_n = is_li && !is_lj ? lt : lt2;
        // refills: li's opening at cap_n + 1, lj's unit at e_n - 1 (clamped reads on every lane)
        const bool rj = is_lj && !is_li;
        const int ia = is_li ? min(cap_n + 2, hi) : max(e_n - 1, 0);
        const int ib = is_li ? min(cap_n + 1, hi) : max(e_n - 2, 0);
        const double r0 = G[ia], r1 = G[ib], r2 = H[ia];
        if (is_li) {
            hn = hn2;
            gn = gn2;
        }
        hn2 = is_li ? (cap_n + 1 < hi ? r2 : kInf) : hn2;
        gn2 = is_li ? (cap_n + 1 < hi ? r0 - r1 : kInf) : gn2;
        lt2_n = rj ? (e_n - 1 > lo ? r0 - r1 : -kInf) : lt2_n;
        cap = cap_n;
        e = e_n;
        lt = lt_n;
        lt2 = lt2_n;
        HALDA_SCANPROF(2, "v"(lt), "v"(gn), "v"(e));
        // lam after the event (its reduction needs no LDS value: it overlaps the broadcast of d)
        const int need_n = swap ? 0 : need - 1;
        const double lam_n = sg.max_f64(lt_n);
        const int lj_n = sg.highest(lt_n == lam_n);
        HALDA_SCANPROF(3, "v"(lam_n), "v"(lj_n));
        S += swap ? d - lam : d;
        need = need_n;
        lam = need_n == 0 ? lam_n : -kInf;
        lj = need_n == 0 ? lj_n : -1;
        T = Te;
        const double v = kc * T + S;
        const bool imp = (need == 0) & (v < best);
        best = imp ? v : best;
        bestE = imp ? e : bestE;
        HALDA_SCANPROF(4, "v"(best), "v"(bestE));
    }
    HALDA_SCANPROF(9, "v"(best));
    nodes += events;
    HALDA_KSTAMP(5);
    if constexpr (SG::S == 16) {
        if (part > 1) {  // a helper: its result for part 1 (it posts the flag itself)
            const int h = part - 2;
            if (act && bestE >= 0) sp.ar->alt_e[h][lane] = bestE;
            if (lane == 0) sp.ar->alt_best[h] = bestE >= 0 ? best : kInf;
            wave_sync();
            return true;
        }
        if (part == 1) {  // the helpers' parts in ascending T, each kept only when strictly better
            for (int h = 0; h < sp.n_parts - 1; ++h) {
                while (__hip_atomic_load(&sp.ar->flag[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
                    __builtin_amdgcn_s_sleep(1);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                const double ab = sp.ar->alt_best[h];
                if (ab < best) {
                    best = ab;
                    bestE = act ? sp.ar->alt_e[h][lane] : 0;
                }
            }
        }
    }
    HALDA_SCANPROF(10, "v"(best), "v"(bestE));
#ifdef HALDA_STAMPS
    if (sp.prof && lane == 0 && act) {
        unsigned long long *o = sp.prof + 16 * (sg.base / 16);
        for (int t = 0; t < 11; ++t) o[t] = pa[t];
        o[15] = (unsigned long long)events;
    }
#endif
#undef HALDA_SCANPROF
    if (bestE >= 0) {  // a capped optimum beat the unconstrained allocation's own T
        if (act) w.st0[lane] = bestE;
    }
    wave_sync();
    return true;
}

// Part 1's publication for the helpers of a split scan: the leaf ranges, phase 0's s_inf and bound.
__device__ inline void split_publish(SplitArea *ar, int lane, bool act, int lo, int hi, double s_inf, double best0,
                                     int lo_sum, int capsum) {
    if (act) {
        ar->lo[lane] = lo;
        ar->hi[lane] = hi;
    }
    if (lane == 0) {
        ar->s_inf = s_inf;
        ar->best0 = best0;
        ar->lo_sum = lo_sum;
        ar->capsum = capsum;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) __hip_atomic_store(&ar->pub, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Phase 0 of a k > 1 instance: the unconstrained greedy exchange from e = lo (rounds: the smallest next
// increment wins and keeps every one still beating the runner-up); e ends at the allocation.
// Every round either takes at least one layer or stops: a row that is not checked yet (the optimistic
// k-slot part 1's helper runs this before the leaf checks' verdict) may hold an infinite entry inside
// its finite ends, whose increments are inf or NaN; no finite increment left, or a run of length 0,
// ends the loop with the allocation incomplete, and that row's failed leaf check (contiguity) sends
// the fleet to the table launch before anyone uses it. (A FieldRec row cannot have such a gap: its
// feasible n-interval only shrinks as w grows, so an infeasible w stays infeasible above.)
template <class SG>
__device__ inline void phase0_greedy(const double *Gall, int RS, int need, const SG &sg, bool act, int hi, int &e) {
    const int lane = sg.sl;
    const double *G = Gall + int64_t(act ? lane : 0) * RS;
    double inc = act && e < hi ? G[e + 1] - G[e] : kInf;
    while (need > 0) {
        const double bv = sg.min_f64(inc);
        if (!(bv < kInf)) break;  // no device can take a layer (or NaN increments): leave it to the checks
        const int win = sg.lowest(inc == bv);
        const double rv = lane == win ? kInf : inc;
        const double m2 = sg.min_f64(rv);
        const int d2 = sg.lowest(rv == m2);
        const int t = take_run(Gall + int64_t(win) * RS, sg.bcast(e, win), sg.bcast(hi, win), need, m2, win < d2, sg);
        if (t <= 0) break;
        if (lane == win) {
            e += t;
            inc = e < hi ? G[e + 1] - G[e] : kInf;
        }
        need -= t;
    }
}

// The leaf checks of one row (lane = device): its finite range [lo, hi] (cnt entries), G convex on it
// within the 1e-12 tolerance (ok), H nondecreasing on it (mono). The caller's lo / hi / cnt / ok / mono
// start at R1 / -1 / 0 / true / true.
__device__ inline void leaf_scan(const double *G, const double *H, int R1, bool act, int &lo, int &hi, int &cnt,
                                 bool &ok, bool &mono) {
    // The row in chunks of 8 entries, the chunk's 16 LDS reads issued together (one LDS latency per
    // chunk, not one per entry; a prefetch of the next chunk measured no faster and cost the k-slot
    // kernel 5 VGPRs). No chain between entries: each entry is checked against its two predecessors
    // (g1, g2; d1 = g1 - g2), which in a contiguous finite range are the sequential scan's prev / dprev,
    // bit for bit; a gap in the range fails the contiguity test at the end, as the sequential scan's
    // "hi == e - 1" fails at the entry after it.
    if (act) {
        double gc[8], hc[8];
        auto load = [&](int e0, double (&g)[8], double (&h)[8]) {
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int e = min(e0 + t, R1 - 1);
                g[t] = G[e];
                h[t] = H[e];
            }
        };
        double g1 = kInf, d1 = -kInf, h1 = -kInf;
        bool f1 = false, f2 = false;
        for (int e0 = 0; e0 < R1; e0 += 8) {
            load(e0, gc, hc);
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int e = e0 + t;
                const double g = gc[t], h = hc[t];
                const bool fin = e < R1 && g < kInf;
                const double d = g - g1;
                const bool conv = !(fin && f1 && f2) || d >= d1 - 1e-12 * fmax(1.0, fabs(g));
                ok = ok && conv;
                mono = mono && (!fin || h >= (f1 ? h1 : -kInf));
                lo = fin ? min(lo, e) : lo;
                hi = fin ? e : hi;
                cnt += fin ? 1 : 0;
                g1 = g;
                d1 = d;
                h1 = h;
                f2 = f1;
                f1 = fin;
            }
        }
        ok = ok && (cnt == 0 || cnt == hi - lo + 1);
    }
}

// Every device of the segment has a finite first and last entry (segment-uniform).
template <class SG>
__device__ inline bool leaf_ends_finite(const double *G, int R1, bool act, const SG &sg) {
    return !sg.any(act && !(G[0] < kInf && G[R1 - 1] < kInf));
}

// k > 1 for fleets of at most 64 devices with convex leaves and nondecreasing cycle times (every
// instance the reference builds): lane = device, the leaf scan and the phase-0 greedy exchange in
// registers (the same choices as leaf_ranges + greedy_alloc: smallest increment first, ties to the
// lowest device, runs taken while they beat the runner-up), then the incremental threshold scan.
// Returns 1 solved (st0 = allocation), 0 infeasible, -1 not applicable (the table DP below runs).
template <class SG>
__device__ int dp_pass_lanes(const WaveCtx &w, const Inst &I, const SG &sg, int64_t &nodes,
                             unsigned long long *stamp = nullptr, const ScanSplit sp = ScanSplit{}) {
    const int M = I.M, R1 = I.R1, RS = I.RS;
    const int lane = sg.sl;
    const bool act = lane < M;
#ifdef HALDA_STAMPS  // diagnostic build (tools/scan_prof.py): entry time, leaf scan, checks, phase 0
    unsigned long long lp_t0 = __builtin_amdgcn_s_memtime(), lp_t1 = 0, lp_t2 = 0, lp_t3 = 0;
#endif
    const double *G = w.G + int64_t(act ? lane : 0) * RS, *H = w.H + int64_t(act ? lane : 0) * RS;
    int lo = R1, hi = -1, cnt = 0;
    bool ok = true, mono = true;
    // part 1 of a split scan whose rows are finite at both ends takes them as [0, R1 - 1] and goes on
    // at once: another wave checks them meanwhile (kslot_check) and the verdict is awaited before this
    // returns (a failed check returns -1, as the check here would have); the helper makes phase 0
    const bool opt = sp.part == 1 && sp.opt && leaf_ends_finite(G, R1, act, sg);
    if (opt) {
        if (act) {
            lo = 0;
            hi = R1 - 1;
            cnt = R1;
        }
    } else {
        leaf_scan(G, H, R1, act, lo, hi, cnt, ok, mono);
    }
    auto done = [&](int r) {  // an optimistic part 1 returns the helper's verdict on its rows first
        if constexpr (SG::S == 16) {
            if (opt) {
                while (sg.any(__hip_atomic_load(&sp.ar->verdict, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0))
                    __builtin_amdgcn_s_sleep(1);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                if (sp.ar->verdict != 1) return -1;
            }
        }
        return r;
    };
#ifdef HALDA_STAMPS
    asm volatile("" ::"v"(ok), "v"(mono), "v"(cnt), "v"(lo), "v"(hi));
    lp_t1 = __builtin_amdgcn_s_memtime();
#endif
    if (sg.any(act && (!ok || !mono))) return -1;
    if (sg.any(act && cnt == 0)) return 0;
#ifdef HALDA_STAMPS
    lp_t2 = __builtin_amdgcn_s_memtime();
    if (stamp) stamp[0] = __builtin_amdgcn_s_memtime();  // leaf scan done
#else
    (void)stamp;
#endif
    LeafInfo li;
    li.convex = true;
    li.mono = true;
    li.empty = false;
    li.lo_sum = sg.sum_i(act ? lo : 0);
    li.cap = sg.sum_i(act ? hi - lo : 0);
    li.my_lo = act ? lo : 0;
    li.my_hi = act ? hi : -1;
    int need = (R1 - 1) - li.lo_sum;
    if (need < 0 || need > li.cap) return done(0);
    // phase 0: unconstrained greedy exchange -- by the helper wave for an optimistic part 1 (it publishes
    // s_inf, the bound and the allocation in st0; the scan awaits them before its first event)
#ifdef HALDA_STAMPS
    auto prof_rec = [&]() {
        lp_t3 = __builtin_amdgcn_s_memtime();
        if (sp.prof && lane == 0 && act) {
            unsigned long long *o = sp.prof + 16 * (sg.base / 16);
            o[11] = lp_t1 - lp_t0;
            o[12] = lp_t2 - lp_t1;
            o[13] = lp_t3 - lp_t2;
            o[14] = lp_t0;
        }
    };
#endif
    if (opt) {
#ifdef HALDA_STAMPS
        prof_rec();
#endif
        LeafInfo lf = li;
        nodes = 1;
        kc_scan_incremental(w, I, sg, 0.0, 0.0, nodes, lf, ScanSplit{sp.part, sp.n_parts, sp.ar, true, true
#ifdef HALDA_STAMPS
                                                                     , sp.prof
#endif
                                                                     , sp.cut8});
        wave_sync();
        return done(1);
    }
    int e = act ? lo : 0;
    phase0_greedy(w.G, RS, need, sg, act, hi, e);
    const double s_inf = sg.sum_f64(act ? G[e] : 0.0);
    const double hmax = sg.max_f64(act ? fmax(0.0, H[e]) : 0.0);
    if (act) w.st0[lane] = e;
    nodes = 1;
#ifdef HALDA_STAMPS
    asm volatile("" ::"v"(e));
    prof_rec();
    if (stamp) stamp[1] = __builtin_amdgcn_s_memtime();  // phase-0 greedy done
#endif
    if constexpr (SG::S == 16) {
        if (sp.part == 1)  // the helpers start from here (kslot_helper)
            split_publish(sp.ar, lane, act, lo, hi, s_inf, I.kc * hmax + s_inf, li.lo_sum, li.cap);
    }
    kc_scan_incremental(w, I, sg, s_inf, I.kc * hmax + s_inf, nodes, li, sp);
    wave_sync();
    return done(1);
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
    // gated: only flagged work can be here -- k = 1 hand-backs (no k > 1 or wide instance in the batch), or
    // the k > 1 instances the screen flagged (the k > 1 launch of launch())
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



enum { K1_OK = 0, K1_INFEASIBLE = 1, K1_FALLBACK = 2 };

__device__ inline double shfl_f64(double v, int src) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = __shfl(int(uint32_t(u)), src), hi = __shfl(int(uint32_t(u >> 32)), src);
    return __builtin_bit_cast(double, (uint64_t(hi) << 32) | lo);
}

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
// kClamp = false: nn is nL or nU itself, which needs no clamp (when nL > nU the split fails whatever the
// tries give)
template <bool kClamp = true>
__device__ inline void rec_try(const FieldRec &r, double aw, double pv, double pvo, int w, int nn, int nL, int nU,
                               double &best, int &bn) {
    if constexpr (kClamp) nn = min(max(nn, nL), nU);
    const int sc = max(0, w - (r.cls == 3 ? nn : 0) + r.Kset), t = max(0, nn + r.Kvram);  // kNoRow: 0
    double g = aw;
    g = g + r.b * double(nn);
    // the class slack's term, priced pvo = (own ? pv : +0): without a class slack it adds +0 * sc = +0, which
    // leaves g's bits unchanged (g is never -0: aw = alpha w >= +0) -- dev_cost's select, without the
    // per-try select
    g = g + pvo * double(sc);
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
    const double pvo = rec_own(r) ? pv : 0.0;
    double best = kInf;
    int bn = -1;
    rec_try<false>(r, aw, pv, pvo, w, nL, nL, nU, best, bn);
    rec_try<false>(r, aw, pv, pvo, w, nU, nL, nU, best, bn);
    const bool hc = r.cls == 3 && r.Kset != kNoRow, hv = r.Kvram != kNoRow;
    if (!kUniform || hc) rec_try(r, aw, pv, pvo, w, hc ? w + r.Kset : nL, nL, nU, best, bn);  // class-slack kink
    if (!kUniform || hv) rec_try(r, aw, pv, pvo, w, hv ? -r.Kvram : nL, nL, nU, best, bn);     // VRAM kink
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
    const double pvo = rec_own(r) ? pv : 0.0;
    double best = kInf;
    int bn = -1;
    rec_try<false>(r, aw, pv, pvo, w, nL, nL, nU, best, bn);
    rec_try<false>(r, aw, pv, pvo, w, nU, nL, nU, best, bn);
    const bool ok = okI & (bn >= 0) & !rec_nanx(r);
    if (ok) {
        g = best;
        n = bn;
        rec_slacks(r, w, bn, s);
    }
    return ok;
}
// split_full at w = 2 (the greedy's first increment): 0 <= nL <= n <= nU <= 2, so the three tries
// n = 0, 1, 2 (clamped to [nL, nU]) cover every candidate split_full tries (its kinks clamp into the
// same range) with the same cost expression and tie rule: the same minimum and least minimiser, one
// try fewer than split_full's four.
__device__ inline bool split_second(const FieldRec &r, int w, double &g, int &n, int s[4]) {
    if (w != 2) return split_full(r, w, g, n, s);
    int nL, nU;
    const bool okI = rec_interval(r, w, nL, nU);
    const double pv = rec_pv(r), aw = r.alpha * double(w);
    const double pvo = rec_own(r) ? pv : 0.0;
    double best = kInf;
    int bn = -1;
    rec_try(r, aw, pv, pvo, w, 0, nL, nU, best, bn);
    rec_try(r, aw, pv, pvo, w, 1, nL, nU, best, bn);
    rec_try(r, aw, pv, pvo, w, 2, nL, nU, best, bn);
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
    const double pvo = rec_own(r) ? pv : 0.0;
    double best = kInf;
    int bn = -1;
    rec_try(r, aw, pv, pvo, w, n_prev, nL, nU, best, bn);
    rec_try(r, aw, pv, pvo, w, n_prev + 1, nL, nU, best, bn);
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
        const bool fb = split_second(d, wlo + 1, gb, nb, sb);
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
//
// kScreen (halda_solve_k1_settled_kernel: no screen launch before it): the screen's verdict on this
// instance rides the same round trips -- the equality row's extent and bounds with round trip 1, its
// entries with round trip 2 (the w lower bounds are round trip 1's) -- and is decided right after round
// trip 2 by the screen's own rules and precedence (screen_group: a non-HALDA equality row, then bound
// infeasibility, then a table beyond the launches' slices, then c[C] > 0 for the k > 1 launch). An
// instance the screen would not class CLS_K1 gets the screen's outputs (status / cls / the k > 1 flag)
// and 3 is returned; sc->screened says whether that point was reached (a return 2 before it leaves the
// screen to the caller).
struct K1Screen {
    int mmax, r1max, tab, tab_kc;
    int *gen_flag;
    int launch_id;
    uint8_t *cls;
    const halda_result *Rz;
    bool screened;
};

template <bool kScreen = false>
__device__ int decode_k1(const halda_batch &B, const WaveCtx &w, unsigned char *scol_raw, unsigned char *sval_raw,
                         Inst &I, int lane, Dev &d, int &sumlo, K1Screen *sc = nullptr) {
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
    // the equality row's rhs W and c[C] (the caller has only the header): in this round trip too
    I.Wd = B.row_ub[I.ro + I.m - 1];
    I.kc = B.c[co + I.iC];
    I.W = int(I.Wd);
    int eqs = 0, eqe = 0;
    double Wl = 0.0;
    if constexpr (kScreen) {  // the equality row's extent and lower bound (screen_group's round trip 2)
        eqs = I.rp[I.m - 1];
        eqe = I.rp[I.m];
        Wl = B.row_lb[I.ro + I.m - 1];
    }
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

    // the screen's verdict: everything but the equality row's entries is in (round trip 1), so it is
    // decided here, before round trip 2 is issued, as far as it goes -- in screen_group's precedence: UNSUPPORTED (equality row),
    // INFEASIBLE (w lower bounds), TOO_LARGE (the launches' slices), CLS_GEN (c[C] > 0) -- and only a
    // scalar code and the row's start are kept; the entries come with the first cycle half below
    // (screen_group's round trip 3), when the capacity rows' registers are free
    int pre = 0, eqb = 0;  // pre: 0 a k = 1 candidate, else the HALDA_STATUS_* / -100 - CLS_GEN verdict
    if constexpr (kScreen) {
        const bool eq_ext = eqe - eqs == M;
        eqb = eq_ext ? eqs : 0;
        const bool lb_inf = wave_or(act && (int(ceil(lbv[0])) > I.W || lbv[0] < 0.0)) != 0;
        if (!(Wl == I.Wd) || !(I.Wd >= 0.0 && I.Wd < 1e6 && I.Wd == floor(I.Wd)) || !eq_ext) {
            pre = HALDA_STATUS_UNSUPPORTED;
        } else if (lb_inf || sumlo > I.W) {
            pre = HALDA_STATUS_INFEASIBLE;
        } else {
            const int R1 = I.W - sumlo + 1;
            const bool kc = I.kc > 0.0;
            if (R1 > sc->r1max || int64_t(M) * odd_stride(R1) > (kc ? sc->tab_kc : sc->tab)) pre = HALDA_STATUS_TOO_LARGE;
            else if (kc) pre = -100 - CLS_GEN;
        }
    }
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
    auto screen_verdict = [&](int ecol, double eval) -> bool {
        sc->screened = true;
        int st = 0, v = CLS_K1;
        if (pre == HALDA_STATUS_UNSUPPORTED || wave_or(act && (ecol != lane || eval != 1.0))) st = HALDA_STATUS_UNSUPPORTED;
        else if (pre == -100 - CLS_GEN) v = CLS_GEN;
        else st = pre;
        if (st || v != CLS_K1) {
            if (lane == 0) {
                sc->cls[I.inst] = uint8_t(st ? CLS_DONE : v);
                if (st) write_done(*sc->Rz, I.inst, st, 0);
                if (v == CLS_GEN) *sc->gen_flag = sc->launch_id;  // the k > 1 launch of this batch has work
            }
            return true;
        }
        if (lane == 0) sc->cls[I.inst] = CLS_K1;  // (a hand-back below rewrites it)
        return false;
    };
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
        if constexpr (kScreen) {
            if (h == 0) {
                const int ei = eqb + li;  // (row 0's entries when the extent is wrong: read, then rejected)
                const int c0 = B.col_idx[ei];
                const double v0 = B.val[ei];
                stage_wait();
                if (screen_verdict(act ? c0 : lane, act ? v0 : 1.0)) return 3;
            }
        }
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

// The compact record (halda_sweep.hpp's FieldRec) whose dev() is exactly d, if there is one: its
// coefficients read back from d, its class from the one class slack open to W, its GPU flag from n's
// bound; then every field of dev() is compared with d's (doubles bit for bit).
__device__ inline int same_bits(double a, double b) { return __double_as_longlong(a) == __double_as_longlong(b); }

__device__ inline bool rec_of_dev(const Dev &d, int W, FieldRec &r) {
    r.alpha = d.cw;
    r.b = d.cn;
    r.p_bp = d.cs0;
    r.p_b = d.cs1;
    r.cst = -d.rhs1;
    r.W = W;
    r.gpu = W > 0 && d.nhi == W;
    r.cls = W <= 0 ? 0 : d.shi[0] == W ? 1 : d.shi[1] == W ? 2 : d.shi[2] == W ? 3 : 0;
    r.Kset = r.cls == 1 ? d.Ks[0] : r.cls == 2 ? d.Ks[1] : r.cls == 3 ? d.Ks[2] : kNoRow;  // selects: no scratch
    r.Kvram = d.Ks[3];
    const Dev e = r.dev();
    int ok = same_bits(e.cw, d.cw) & same_bits(e.cn, d.cn) & same_bits(e.cs0, d.cs0) & same_bits(e.cs1, d.cs1) &
              same_bits(e.cs2, d.cs2) & same_bits(e.cs3, d.cs3) & same_bits(e.r1w, d.r1w) &
              same_bits(e.r2w, d.r2w) & same_bits(e.rhs1, d.rhs1) & same_bits(e.rhs2, d.rhs2);
    ok &= (e.wlo == d.wlo) & (e.whi == d.whi) & (e.nlo == d.nlo) & (e.nhi == d.nhi);
#pragma unroll
    for (int j = 0; j < 4; ++j)
        ok &= (e.slo[j] == d.slo[j]) & (e.shi[j] == d.shi[j]) & (e.us[j] == d.us[j]) & (e.vs[j] == d.vs[j]) &
              (e.Ks[j] == d.Ks[j]);
#pragma unroll
    for (int j = 0; j < 2; ++j) ok &= (e.uf[j] == d.uf[j]) & (e.vf[j] == d.vf[j]) & (e.Kf[j] == d.Kf[j]);
    return ok;
}

// The greedy and the output of a decoded k = 1 instance on its compact records (the greedy hands back
// its split at the returned e, so the output needs no split of its own).
__device__ inline void k1_finish(const halda_result &Rz, uint8_t *cls, const Inst &I, int lane, int *hb_flag,
                                 int launch_id, const FieldRec &rec, int sumlo) {
    int e = 0, rounds = 0, nE = 0;
    double gE = 0.0;
    const int rc = k1_alloc(rec, I.M, I.W - sumlo, Wave(lane), e, rounds, gE, nE);
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
    const auto &d = rec.core();
    double g = 0.0, H = 0.0;
    if (lane < I.M) {
        const int wl = rec_wlo(d) + e;
        double P, Q;
        int n = 0, s[4] = {0, 0, 0, 0};
        g = gE;  // split_full's values at wl (k1_alloc)
        n = nE;
        rec_slacks(d, wl, n, s);
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
}

// One k = 1 instance (lane = device) from decode to x; hands the instance to the
// general kernel (cls = CLS_GEN) when the fast path does not apply.
template <bool kScreen = false>
__device__ void solve_k1(const halda_batch &B, const halda_result &Rz, uint8_t *cls, const WaveCtx &w,
                         unsigned char *scol, unsigned char *sval, Inst I, int lane, int *hb_flag,
                         int launch_id, K1Screen *sc = nullptr) {
    HALDA_STAMP(0);
    Dev d = {};
    int sumlo = 0;
    const int fast = decode_k1<kScreen>(B, w, scol, sval, I, lane, d, sumlo, sc);
    HALDA_PSTAMP(1);
    if (kScreen && fast == 3) {  // the screen's verdict is written (not a k = 1 fast-path instance)
        wave_sync();
        return;
    }
    if (kScreen && fast == 2 && !sc->screened) {
        // this shape leaves decode_k1 before its screen point: the screen's own code on this one instance
        wave_sync();
        if (screen_one(B, Rz, cls, I.inst, lane, sc->mmax, sc->r1max, sc->tab, sc->tab_kc, sc->gen_flag, launch_id) !=
            CLS_K1)
            return;  // settled or classed for the general launches
    }
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
    // the decoded records in the fused sweep's compact form when every device's record is exactly
    // what that form expands to (the reference lowering's shape): the greedy and the output run the
    // register sweep's specialised arithmetic (the same candidates and tie rule: the same bits;
    // 47.6 -> 43.9 us per C3 launch against the greedy on the generic decoded records)
    FieldRec r;
    const bool same = rec_of_dev(d, I.W, r);
    if (__ballot(lane < I.M && !same) == 0) {
        k1_finish(Rz, cls, I, lane, hb_flag, launch_id, r, sumlo);
    } else {
        // another record shape (a valid HALDA MILP the reference lowering does not write): the k = 1
        // general launch takes it. Greedy on the generic records here instead: 3.7 us slower per C3
        // launch (the second k1_alloc instantiation costs registers), for instances that do not occur.
        wave_sync();
        if (lane == 0) {
            cls[I.inst] = CLS_GEN1;
            *hb_flag = launch_id;
        }
    }
    HALDA_STAMP(6);
}

// One k = 1 instance of the fast path from its header (decode_k1 loads W and c[C] with its first round
// trip).
__device__ inline void k1_instance(const halda_batch &B, const halda_result &Rz, uint8_t *cls, const WaveCtx &w,
                                   unsigned char *scol, unsigned char *sval, int lane, int *hb_flag, int launch_id,
                                   int64_t inst, int N, int m, int64_t co, int64_t ro, int64_t cs) {
    Inst I;
    I.inst = int(inst);
    I.m = m;
    I.M = (N - 1) / 7;
    I.iC = 7 * I.M;
    I.invM = 1.0f / float(I.M);
    I.co = co;
    I.ro = ro;
    I.rp = B.row_ptr + cs;
    I.Wd = 0.0;
    I.W = 0;
    I.kc = 0.0;
    solve_k1(B, Rz, cls, w, scol, sval, I, lane, hb_flag, launch_id);
}

// Screen: four waves per workgroup, each screening kScreenPer consecutive instances.
__global__ __launch_bounds__(256) void halda_screen_kernel(halda_batch B, halda_result Rz, uint8_t *cls, int mmax,
                                                           int r1max, int tab, int tab_kc,
                                                           const uint8_t *settled, int *gen_flag, int launch_id) {
    const int lane = threadIdx.x & 63;
    const int64_t i0 = (int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6)) * kScreenPer;
    if (i0 >= B.n_inst) return;
    ScreenOut so;
    screen_group(B, Rz, cls, i0, lane, mmax, r1max, tab, tab_kc, so, settled, gen_flag, launch_id);
}

// The k = 1 kernel of a settled batch (halda_solve_batch_device_settled) with no screen launch before
// it: the caller's settled instances get the screen's INFEASIBLE outputs lane-parallel (their rows are
// never read), and every other instance is screened by its own wave on the way -- the screen's verdict
// rides decode_k1's round trips (kScreen), so a k = 1 instance costs no round trip beyond the fast
// path's own. What the screen would not class CLS_K1 is written as the screen writes it (status, or
// cls + the k > 1 launch's flag) for the general launches behind this one.
__global__ __launch_bounds__(64, HALDA_K1_WAVES_PER_SIMD) void halda_solve_k1_settled_kernel(
    halda_batch B, halda_result Rz, uint8_t *cls, int mmax, int *hb_flag, int launch_id, const uint8_t *settled,
    int *gen_flag, int r1max, int tab, int tab_kc) {
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
    K1Screen sc{mmax, r1max, tab, tab_kc, gen_flag, launch_id, cls, &Rz, false};
    const int S = gridDim.x;
    const int vb = blockIdx.x;  // (an XCD-grouped map, consecutive instances on one XCD: -2 % fetch, no faster)
    // the screen's outputs for the settled instances (screen_group: hint), 64 consecutive instances per
    // wave and pass, lane = instance: whole-line stores (the strided walk below would scatter them one
    // line each; a stretch of n / gridDim instances per wave left partial lines: +5 MB of writes at C3)
    for (int64_t i = int64_t(vb) * 64 + lane; i - lane < B.n_inst; i += int64_t(64) * S)
        if (i < B.n_inst && settled[i]) {
            cls[i] = CLS_DONE;
            write_done(Rz, int(i), HALDA_STATUS_INFEASIBLE, 0);
        }
    for (int64_t base = vb; base < B.n_inst; base += int64_t(64) * S) {
        // lane * S formed again on every pass (asm: not hoisted out of the loop): held across the
        // instances it was the kernel's one spill, 512 B of scratch written and read per wave
        int ls;
        asm volatile("v_mul_lo_u32 %0, %1, %2" : "=v"(ls) : "v"(lane), "s"(S));
        const int64_t mine = base + ls;
        const bool in = mine < B.n_inst;
        const bool done = in && settled[in ? mine : 0] != 0;
        uint64_t todo = __ballot(in && !done);
        while (todo) {
            const int bit = __builtin_ctzll(todo);
            todo &= todo - 1;
            const int64_t i = base + int64_t(bit) * S;
            const int N = B.n_cols[i], m = B.n_rows[i];
            const int M = N >= 1 ? (N - 1) / 7 : 0;
            sc.screened = false;
            if (N < 1 || (N - 1) % 7 != 0 || m < 1 || M < 1 || M > min(mmax, kK1MaxM)) {
                // not a k = 1 fast-path shape: the screen's own code decides (and writes) it
                if (screen_one(B, Rz, cls, i, lane, mmax, r1max, tab, tab_kc, gen_flag, launch_id) == CLS_K1 &&
                    lane == 0) {
                    cls[i] = CLS_GEN1;  // (M > 64 is classed CLS_GEN1 by the screen itself)
                    *hb_flag = launch_id;
                }
                wave_sync();
                continue;
            }
            Inst I;
            I.inst = int(i);
            I.m = m;
            I.M = M;
            I.iC = 7 * M;
            I.invM = 1.0f / float(M);
            I.co = B.col_off[i];
            I.ro = B.row_off[i];
            I.rp = B.row_ptr + B.csr_off[i];
            I.Wd = 0.0;
            I.W = 0;
            I.kc = 0.0;
            solve_k1<true>(B, Rz, cls, w, scol, sval, I, lane, hb_flag, launch_id, &sc);
        }
    }
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
            const int64_t i = base + int64_t(bit) * S;
            k1_instance(B, Rz, cls, w, scol, sval, lane, hb_flag, launch_id, i, B.n_cols[i], B.n_rows[i],
                        B.col_off[i], B.row_off[i], B.csr_off[i]);
        }
    }
}
