/*
 * halda_exact.c — TEST INFRASTRUCTURE ONLY (oracle). Never linked into, or
 * called by, the product path (distilp_amd / libhalda). Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Exact CPU solver for one fixed-k HALDA MILP, given in the dense form the
 * reference hands to scipy.optimize.milp (src/distilp/solver/halda_p_solver.py
 * :299-346): A = [A_ub ; A_eq] (row-major, m x n), row bounds bl/bu, objective
 * c, column bounds lb/ub, integrality. It is independent of the GPU kernel: it
 * identifies rows by their nonzero pattern, enumerates EVERY integer (w_i, n_i)
 * pair of every device by brute force, and runs a 2-best min-plus DP so that it
 * also reports the objective of the best *distinct* second solution (the
 * uniqueness margin the parity tests use).
 *
 * Why this is exact: the stall variables z_i occur
 * only in the two cycle rows of device i, so for fixed integer columns the
 * least feasible cycle time is C >= max(P_i, (P_i + Q_i)/2) with
 * P_i = row1_i.x - rhs1_i, Q_i = row2_i.x - rhs2_i; every slack (s1,s2,s3,t)
 * has a positive cost in the objective and in the cycle rows, so it sits at
 * the least integer its capacity rows allow. What remains is a separable
 * choice of (w_i, n_i) under sum_i w_i = W plus a max-coupling through C with
 * weight c[C] = k-1, solved by a DP over sum(w) for every candidate value T of
 * max_i H_i (pruned once (k-1)T + min sum g exceeds the running second best).
 *
 * The slack rule s = ceil(need - eps) treats a capacity row as satisfied
 * within eps layers, mirroring HiGHS's primal feasibility tolerance
 * (1e-7 on its scaled rows, scipy 1.15.3 / HiGHS 1.8.0).
 *
 * Parity pinned by the JSON goldens under tests/golden (generated from the reference + HiGHS).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define EX_OK 0
#define EX_INFEASIBLE 2
#define EX_UNSUPPORTED (-1)
#define EX_NOMEM (-2)

typedef struct {
    int slack; /* 0..3 = s1,s2,s3,t ; -1 = no slack (pure w/n row) */
    double aw, an, beta, rhs;
} cap_row;

typedef struct {
    int ncap;
    cap_row cap[8];
    int have1, have2;
    double r1[6], r2[6], rhs1, rhs2; /* cycle rows restricted to w,n,s1,s2,s3,t */
} device_rows;

typedef struct {
    double g, h; /* objective contribution, least cycle time */
    int feasible;
    int s[4];
} pair_eval;

static int is_int(double v) { return isfinite(v) && v == floor(v); }

/* top-2 option record for one device & one w at a threshold */
typedef struct {
    double g[2];
    int n[2];
    int cnt;
} top2;

/* DP cell: two best distinct partial solutions */
typedef struct {
    double v[2];
    int w[2], opt[2], prev[2];
    int cnt;
} cell;

static void cell_push(cell *c, double v, int w, int opt, int prev) {
    if (c->cnt < 2) {
        int pos = c->cnt;
        if (pos == 1 && v < c->v[0]) {
            c->v[1] = c->v[0]; c->w[1] = c->w[0]; c->opt[1] = c->opt[0]; c->prev[1] = c->prev[0];
            pos = 0;
        }
        c->v[pos] = v; c->w[pos] = w; c->opt[pos] = opt; c->prev[pos] = prev;
        c->cnt++;
        return;
    }
    if (v < c->v[0]) {
        c->v[1] = c->v[0]; c->w[1] = c->w[0]; c->opt[1] = c->opt[0]; c->prev[1] = c->prev[0];
        c->v[0] = v; c->w[0] = w; c->opt[0] = opt; c->prev[0] = prev;
    } else if (v < c->v[1]) {
        c->v[1] = v; c->w[1] = w; c->opt[1] = opt; c->prev[1] = prev;
    }
}

typedef struct {
    int M, W, wmax, nmax;
    pair_eval *pe; /* [M][wmax+1][nmax+1] */
    int *wlo, *whi, *nlo, *nhi;
} problem;

static pair_eval *PE(problem *p, int i, int w, int n) {
    return &p->pe[((size_t)i * (p->wmax + 1) + w) * (p->nmax + 1) + n];
}

/* 2-best DP at threshold T (use_T = 0: no threshold). Returns number of
 * solutions found (0..2); sol_w/sol_n receive them (M entries each). */
static int dp2(problem *p, int use_T, double T, top2 *opts, cell *dp, int *sol_w, int *sol_n, double *sol_g) {
    const int M = p->M, W = p->W;
    const int stride = W + 1;
    /* options per (device, w) */
    for (int i = 0; i < M; i++)
        for (int w = 0; w <= W; w++) {
            top2 *t = &opts[i * stride + w];
            t->cnt = 0;
            if (w < p->wlo[i] || w > p->whi[i]) continue;
            for (int n = p->nlo[i]; n <= p->nhi[i] && n <= p->nmax; n++) {
                pair_eval *e = PE(p, i, w, n);
                if (!e->feasible) continue;
                if (use_T && fmax(0.0, e->h) > T) continue;
                double g = e->g;
                if (t->cnt < 2) {
                    int pos = t->cnt;
                    if (pos == 1 && g < t->g[0]) { t->g[1] = t->g[0]; t->n[1] = t->n[0]; pos = 0; }
                    t->g[pos] = g; t->n[pos] = n; t->cnt++;
                } else if (g < t->g[0]) {
                    t->g[1] = t->g[0]; t->n[1] = t->n[0]; t->g[0] = g; t->n[0] = n;
                } else if (g < t->g[1]) {
                    t->g[1] = g; t->n[1] = n;
                }
            }
        }
    /* stage 0 = empty prefix */
    for (int v = 0; v <= W; v++) dp[v].cnt = 0;
    dp[0].cnt = 1; dp[0].v[0] = 0.0; dp[0].w[0] = -1;
    for (int i = 0; i < M; i++) {
        cell *prev = &dp[(size_t)i * stride], *cur = &dp[(size_t)(i + 1) * stride];
        for (int v = 0; v <= W; v++) {
            cur[v].cnt = 0;
            for (int w = 0; w <= v; w++) {  /* opts hold only w in [lb, ub] */
                top2 *t = &opts[i * stride + w];
                cell *pc = &prev[v - w];
                for (int o = 0; o < t->cnt; o++)
                    for (int r = 0; r < pc->cnt; r++) cell_push(&cur[v], pc->v[r] + t->g[o], w, o, r);
            }
        }
    }
    cell *fin = &dp[(size_t)M * stride + W];
    for (int r = 0; r < fin->cnt; r++) {
        int v = W, rank = r;
        sol_g[r] = fin->v[r];
        for (int i = M - 1; i >= 0; i--) {
            cell *c = &dp[(size_t)(i + 1) * stride + v];
            int w = c->w[rank], o = c->opt[rank];
            sol_w[r * M + i] = w;
            sol_n[r * M + i] = opts[i * stride + w].n[o];
            rank = c->prev[rank];
            v -= w;
        }
    }
    return fin->cnt;
}

static int cmp_double(const void *a, const void *b) {
    double x = *(const double *)a, y = *(const double *)b;
    return (x > y) - (x < y);
}

/* true objective of a full solution */
static double sol_obj(problem *p, double kc, const int *w, const int *n, double *Cout) {
    double gsum = 0.0, hmax = 0.0;
    for (int i = 0; i < p->M; i++) {
        pair_eval *e = PE(p, i, w[i], n[i]);
        gsum += e->g;
        if (e->h > hmax) hmax = e->h;
    }
    if (Cout) *Cout = hmax;
    return kc * hmax + gsum;
}

int halda_exact_solve(int n, int m, const double *A, const double *bl, const double *bu, const double *c,
                      const double *lb, const double *ub, const uint8_t *integ, double eps, double *x_out,
                      double *best_out, double *second_out, int64_t *nodes_out) {
    if (n < 1 || (n - 1) % 7 != 0 || m < 1) return EX_UNSUPPORTED;
    const int M = (n - 1) / 7, iC = 7 * M;
    *nodes_out = 0;
    /* equality row: last row, sum_i w_i = W */
    const double *eq = &A[(size_t)(m - 1) * n];
    if (!(bl[m - 1] == bu[m - 1]) || !is_int(bu[m - 1])) return EX_UNSUPPORTED;
    for (int j = 0; j < n; j++) {
        double want = j < M ? 1.0 : 0.0;
        if (eq[j] != want) return EX_UNSUPPORTED;
    }
    const int W = (int)bu[m - 1];
    if (c[iC] < 0) return EX_UNSUPPORTED;
    for (int j = 6 * M; j < iC; j++)
        if (c[j] != 0.0 || integ[j]) return EX_UNSUPPORTED;
    for (int j = 0; j < 6 * M; j++)
        if (!integ[j]) return EX_UNSUPPORTED;
    /* column bounds */
    int *wlo = calloc(4 * (size_t)(M ? M : 1), sizeof(int));
    if (!wlo) return EX_NOMEM;
    int *whi = wlo + M, *nlo = wlo + 2 * M, *nhi = wlo + 3 * M;
    int slo[4][M ? M : 1], shi[4][M ? M : 1];
    int status = EX_OK;
    for (int i = 0; i < M; i++) {
        wlo[i] = (int)ceil(lb[i]); whi[i] = (int)floor(ub[i]);
        nlo[i] = (int)ceil(lb[M + i]); nhi[i] = (int)floor(ub[M + i]);
        for (int s = 0; s < 4; s++) {
            slo[s][i] = (int)ceil(lb[(2 + s) * M + i]);
            shi[s][i] = (int)floor(ub[(2 + s) * M + i]);
        }
        if (wlo[i] > whi[i] || nlo[i] > nhi[i]) status = EX_INFEASIBLE;
    }
    for (int j = 6 * M; j <= iC; j++)
        if (lb[j] != 0.0) { free(wlo); return EX_UNSUPPORTED; }
    /* classify rows */
    device_rows *dr = calloc(M ? M : 1, sizeof(device_rows));
    if (!dr) { free(wlo); return EX_NOMEM; }
    for (int r = 0; r < m - 1 && status == EX_OK; r++) {
        const double *row = &A[(size_t)r * n];
        if (bl[r] != -INFINITY) { status = EX_UNSUPPORTED; break; }
        if (row[iC] != 0.0) {
            int dev = -1, sign = 0;
            for (int i = 0; i < M; i++)
                if (row[6 * M + i] != 0.0) {
                    if (dev >= 0) { status = EX_UNSUPPORTED; break; }
                    dev = i; sign = row[6 * M + i] > 0 ? 1 : -1;
                    if (fabs(row[6 * M + i]) != 1.0) status = EX_UNSUPPORTED;
                }
            if (dev < 0 || row[iC] != -1.0 || status != EX_OK) { status = EX_UNSUPPORTED; break; }
            for (int j = 0; j < 6 * M; j++)
                if (row[j] != 0.0 && j % M != dev) status = EX_UNSUPPORTED;
            device_rows *d = &dr[dev];
            double *dst = sign > 0 ? d->r1 : d->r2;
            for (int b = 0; b < 6; b++) dst[b] = row[b * M + dev];
            if (sign > 0) { d->have1++; d->rhs1 = bu[r]; } else { d->have2++; d->rhs2 = bu[r]; }
        } else {
            int dev = -1, slack = -1;
            for (int j = 0; j < iC; j++) {
                if (row[j] == 0.0) continue;
                if (j >= 6 * M) { status = EX_UNSUPPORTED; break; }
                int i = j % M, blk = j / M;
                if (dev >= 0 && i != dev) { status = EX_UNSUPPORTED; break; }
                dev = i;
                if (blk >= 2) {
                    if (slack >= 0) { status = EX_UNSUPPORTED; break; }
                    slack = blk - 2;
                }
            }
            if (status != EX_OK) break;
            if (dev < 0) { if (bu[r] < 0) status = EX_INFEASIBLE; continue; }
            device_rows *d = &dr[dev];
            if (d->ncap >= 8) { status = EX_UNSUPPORTED; break; }
            cap_row *cr = &d->cap[d->ncap++];
            cr->slack = slack;
            cr->aw = row[dev];
            cr->an = row[M + dev];
            cr->beta = slack >= 0 ? -row[(2 + slack) * M + dev] : 0.0;
            cr->rhs = bu[r];
            if (slack >= 0 && !(cr->beta > 0)) status = EX_UNSUPPORTED;
        }
    }
    for (int i = 0; i < M && status == EX_OK; i++)
        if (dr[i].have1 != 1 || dr[i].have2 != 1) status = EX_UNSUPPORTED;
    for (int j = 2 * M; j < 6 * M && status == EX_OK; j++)
        if (c[j] < 0) status = EX_UNSUPPORTED;
    if (status == EX_OK) { /* bound infeasibility: sum_i ceil(lb(w_i)) > W (M > W for the reference's lb = 1) */
        long long sumlo = 0;
        for (int i = 0; i < M; i++) sumlo += wlo[i];
        if (sumlo > W) status = EX_INFEASIBLE;
    }
    if (status == EX_OK && M == 0) status = W == 0 ? EX_OK : EX_INFEASIBLE;
    if (status != EX_OK || M == 0) {
        free(dr); free(wlo);
        if (status == EX_OK) { /* empty fleet with W = 0: x = [C = 0] */
            x_out[iC] = 0.0; *best_out = 0.0; *second_out = INFINITY;
        }
        return status;
    }
    /* enumerate all (w, n) pairs of every device */
    problem p = {M, W, W, 0, NULL, wlo, whi, nlo, nhi};
    for (int i = 0; i < M; i++) {
        if (whi[i] > W) whi[i] = W;
        if (nhi[i] > p.nmax) p.nmax = nhi[i];
    }
    if (p.nmax > W) p.nmax = W;
    p.pe = calloc((size_t)M * (W + 1) * (p.nmax + 1), sizeof(pair_eval));
    if (!p.pe) { free(dr); free(wlo); return EX_NOMEM; }
    size_t npairs = 0;
    for (int i = 0; i < M; i++) {
        device_rows *d = &dr[i];
        for (int w = wlo[i]; w <= whi[i]; w++)
            for (int nn = nlo[i]; nn <= nhi[i] && nn <= p.nmax; nn++) {
                pair_eval *e = PE(&p, i, w, nn);
                e->feasible = 1;
                for (int s = 0; s < 4; s++) e->s[s] = slo[s][i];
                for (int q = 0; q < d->ncap && e->feasible; q++) {
                    cap_row *cr = &d->cap[q];
                    double act = cr->aw * w + cr->an * nn - cr->rhs;
                    if (cr->slack < 0) {
                        if (act > eps * fmax(1.0, fabs(cr->rhs))) e->feasible = 0;
                        continue;
                    }
                    double need = ceil(act / cr->beta - eps);
                    if (need > e->s[cr->slack]) {
                        if (need > shi[cr->slack][i]) { e->feasible = 0; break; }
                        e->s[cr->slack] = (int)need;
                    }
                }
                if (!e->feasible) continue;
                for (int s = 0; s < 4; s++)
                    if (e->s[s] > shi[s][i]) e->feasible = 0;
                if (!e->feasible) continue;
                double xv[6] = {w, nn, e->s[0], e->s[1], e->s[2], e->s[3]};
                double g = 0.0, a1 = 0.0, a2 = 0.0;
                for (int b = 0; b < 6; b++) {
                    g += c[b * M + i] * xv[b];
                    a1 += d->r1[b] * xv[b];
                    a2 += d->r2[b] * xv[b];
                }
                double P = a1 - d->rhs1, Q = a2 - d->rhs2;
                e->g = g;
                e->h = Q >= P ? 0.5 * (P + Q) : P;
                npairs++;
            }
    }
    const int stride = W + 1;
    top2 *opts = malloc(sizeof(top2) * (size_t)M * stride);
    cell *dp = malloc(sizeof(cell) * (size_t)(M + 1) * stride);
    int *sw = malloc(sizeof(int) * 6 * (size_t)M);
    double *hs = malloc(sizeof(double) * (npairs + 1));
    if (!opts || !dp || !sw || !hs) {
        free(opts); free(dp); free(sw); free(hs); free(p.pe); free(dr); free(wlo);
        return EX_NOMEM;
    }
    int *sn = sw + 2 * M, *best_w = sw + 4 * M, *best_n = sw + 5 * M;
    const double kc = c[iC];
    double best = INFINITY, second = INFINITY, sg[2];
    int found = 0, cnt;

    /* candidate solutions from one DP run -> running top-2 distinct */
#define CONSIDER(cnt)                                                                  \
    for (int r = 0; r < (cnt); r++) {                                                  \
        double ob = sol_obj(&p, kc, &sw[r * M], &sn[r * M], NULL);                     \
        int same = found && !memcmp(&sw[r * M], best_w, sizeof(int) * M) &&             \
                   !memcmp(&sn[r * M], best_n, sizeof(int) * M);                       \
        if (same) continue;                                                            \
        if (ob < best) {                                                               \
            if (found) second = best;                                                  \
            best = ob; found = 1;                                                      \
            memcpy(best_w, &sw[r * M], sizeof(int) * M);                               \
            memcpy(best_n, &sn[r * M], sizeof(int) * M);                               \
        } else if (ob < second) {                                                      \
            second = ob;                                                               \
        }                                                                              \
    }

    cnt = dp2(&p, 0, 0.0, opts, dp, sw, sn, sg);
    (*nodes_out)++;
    if (cnt == 0) { status = EX_INFEASIBLE; goto done; }
    const double s_inf = sg[0];
    CONSIDER(cnt);
    if (kc > 0) {
        size_t nh = 0;
        for (int i = 0; i < M; i++)
            for (int w = wlo[i]; w <= whi[i]; w++)
                for (int nn = nlo[i]; nn <= nhi[i] && nn <= p.nmax; nn++) {
                    pair_eval *e = PE(&p, i, w, nn);
                    if (e->feasible) hs[nh++] = fmax(0.0, e->h);
                }
        qsort(hs, nh, sizeof(double), cmp_double);
        for (size_t q = 0; q < nh; q++) {
            if (q && hs[q] == hs[q - 1]) continue;
            double T = hs[q];
            if (kc * T + s_inf > second) break; /* nothing at or above T can be top-2 */
            cnt = dp2(&p, 1, T, opts, dp, sw, sn, sg);
            (*nodes_out)++;
            CONSIDER(cnt);
        }
    }
#undef CONSIDER
    /* assemble x */
    {
        double Cmax = 0.0;
        for (int i = 0; i < M; i++) {
            pair_eval *e = PE(&p, i, best_w[i], best_n[i]);
            if (e->h > Cmax) Cmax = e->h;
        }
        for (int i = 0; i < M; i++) {
            pair_eval *e = PE(&p, i, best_w[i], best_n[i]);
            device_rows *d = &dr[i];
            double xv[6] = {best_w[i], best_n[i], e->s[0], e->s[1], e->s[2], e->s[3]};
            double a1 = 0.0, a2 = 0.0;
            for (int b = 0; b < 6; b++) {
                x_out[b * M + i] = xv[b];
                a1 += d->r1[b] * xv[b];
                a2 += d->r2[b] * xv[b];
            }
            double P = a1 - d->rhs1, Q = a2 - d->rhs2;
            x_out[6 * M + i] = Q > P ? 0.5 * (Q - P) : 0.0;
        }
        x_out[iC] = Cmax;
        *best_out = best;
        *second_out = second;
    }
done:
    free(opts); free(dp); free(sw); free(hs);
    free(p.pe); free(dr); free(wlo);
    return status;
}
