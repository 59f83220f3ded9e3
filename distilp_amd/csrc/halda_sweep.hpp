// halda_sweep.hpp -- the whole k-sweep (halda_solve_fleets): the GPU lowering, the fused sweep kernels
// (register, pipelined, table, segment, k-slot) and the CSR path's pick kernel.
// Part of libhalda's single translation unit: included by halda.hip inside its anonymous namespace
// (after halda_solve.hpp); not a standalone header.
#pragma once
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
    double ram, ccpu, cgpu, cuda, metal, swap;  // byte counts: integers below 2^53, so the integer sums and
                                                // differences of the reference are exact in double
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

// load_fields with a 32-bit device index (the table's arrays below 4 GiB: the host checks): each load is
// the array's base in SGPRs plus one shared 32-bit byte offset, no per-field 64-bit address arithmetic
// (the steps kernel: 864 -> 845 VALU per C3 item).
template <class T>
__device__ inline T at32(const T *p, uint32_t boff) {
    return *reinterpret_cast<const T *>(reinterpret_cast<const char *>(p) + boff);
}
__device__ inline DevFields load_fields32(const halda_fleets &F, uint32_t g) {
    const uint32_t o8 = g * 8u;
    DevFields f;
    f.scpu = at32(F.scpu_b1, o8); f.sgpu = at32(F.sgpu_b1, o8); f.Tc = at32(F.T_cpu, o8); f.Tg = at32(F.T_gpu, o8);
    f.tkc = at32(F.t_kvcpy_cpu, o8); f.tkg = at32(F.t_kvcpy_gpu, o8); f.r2v = at32(F.t_ram2vram, o8);
    f.v2r = at32(F.t_vram2ram, o8); f.tcomm = at32(F.t_comm, o8); f.sdisk = at32(F.s_disk, o8);
    f.ram = at32(F.d_avail_ram, o8); f.ccpu = at32(F.c_cpu, o8); f.cgpu = at32(F.c_gpu, o8);
    f.cuda = at32(F.d_avail_cuda, o8); f.metal = at32(F.d_avail_metal, o8); f.swap = at32(F.swap, o8);
    f.cls = at32(F.os_class, g);
    f.flags = at32(F.flags, g);
    return f;
}

// The model as the sweep kernels see it: halda_model plus the uniform quotient (b_in / V) + b_out
// formed once on the host (the same IEEE double operations, -ffp-contract=off: the same bits) instead
// of by every wave.
struct SweepModel : halda_model {
    double bvo;  // (b_in / V) + b_out
};

__host__ __device__ inline double model_bvo(const halda_model &Mo) { return (Mo.b_in / Mo.V) + Mo.b_out; }

__device__ inline DevCoef dev_coef(const halda_model &Mo, const DevFields &F, double bvo) {
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
    o.bcio = bvo * head + F.ccpu;
    const double sd = fmax(1.0, F.sdisk);
    o.p_bp = bp / sd;
    o.p_b = Mo.b_layer / sd;
    o.p_v = cls == 2 ? o.p_b : o.p_bp;
    o.cst = o.xi + F.tcomm;
    return o;
}

__device__ inline DevCoef dev_coef(const halda_model &Mo, const DevFields &F) { return dev_coef(Mo, F, model_bvo(Mo)); }

__device__ inline DevCoef dev_coef(const halda_model &Mo, const halda_fleets &F, int64_t g) {
    return dev_coef(Mo, load_fields(F, g));
}

// Right-hand sides of the capacity rows (halda_p_solver.py:227-277).
__device__ inline double rhs_ram(const DevFields &F, int set, double bcio) {
    if (set == 1) return F.ram - bcio;
    if (set == 2) return F.metal - bcio - F.cgpu;
    return (F.ram + F.swap) - bcio;  // the reference's integer sum, exact
}
__device__ inline double rhs_cuda(const DevFields &F) { return F.cuda - F.cgpu; }
__device__ inline double rhs_metal(const halda_model &Mo, const DevFields &F) {
    const double head = (F.flags & HALDA_DEV_HEAD) ? 1.0 : 0.0;
    return F.metal - F.cgpu - Mo.b_out * head;
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
        const double tl = ((F.c_cpu[g] - F.d_avail_ram[g]) - F.swap[g]) / F.s_disk[g];
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
        const double tl = ((F.c_cpu[g] - F.d_avail_ram[g]) - F.swap[g]) / F.s_disk[g];
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

// FieldRec (the compact device record) and its specialised solve primitives: halda_solve.hpp.

__device__ inline FieldRec field_rec(const SweepModel &Mo, const DevFields &F, int &bad) {
    FieldRec r;
    const DevCoef c = dev_coef(Mo, F, Mo.bvo);
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
    const SweepModel *Mo;
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
    return f.cls != 2 ? ((f.ccpu - f.ram) - f.swap) / f.sdisk : 0.0;
}
__device__ inline double xi_term(const DevFields &f) { return (f.r2v + f.v2r) * ((f.flags & HALDA_DEV_UMA) ? 0.0 : 1.0); }

__device__ inline double kappa_head(const halda_model &Mo, int flags, double scpu, double Tc, double sdisk) {
    double total = f_over_s(Mo.has_f_out && (flags & HALDA_DEV_CPU_RATE), Mo.f_out_b1, scpu);
    total += (Mo.b_in / Mo.V + Mo.b_out) / Tc;
    total += Mo.b_in / (Mo.V * sdisk);
    total += Mo.b_out / sdisk;
    return total;
}

template <class SG, bool kLds = false>
__device__ inline void fleet_offsets_regs(const SweepModel &Mo, const DevFields &mf, int M, const SG &sg, double &tsum,
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
    const int j = sg.sl & 3;
    // the four numerators as register values: a select chain over kernel arguments is otherwise turned
    // into a per-lane vector load from the argument segment (a vector memory wait of its own)
    double n0 = Mo.f_out_b1, n1 = Mo.bvo, n2 = Mo.b_in, n3 = Mo.b_out;
    if constexpr (kLds) {  // the model read from LDS: vector registers
        asm volatile("" : "+v"(n0), "+v"(n1), "+v"(n2), "+v"(n3));
    } else {
        asm volatile("" : "+s"(n0), "+s"(n1), "+s"(n2), "+s"(n3));
    }
    const double num = j == 0 ? n0 : j == 1 ? n1 : j == 2 ? n2 : n3;
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

// SweepArgs.outs: which optional outputs the call wants, in one word the waves read with the first
// kernel-argument line (testing the pointers themselves costs a dependent scalar load each)
constexpr int kOutObk = 1, kOutSt = 2, kOutX = 4, kOutC = 8, kOutXC = kOutX | kOutC, kOutXZ = 16;

struct SweepArgs {
    SweepModel Mo;
    halda_fleets F;
    int n_k;
    int uM;                        // > 0: every fleet has uM devices (dev_off[f] = dev_off[0] + f uM)
    int outs;                      // kOut* bits
    FleetOut out;
    int64_t xstride;
    uint8_t *fflag;  // per fleet: 1 = needs the table launch
    int *hb_flag;
    int launch_id;
    int want;                      // 0: every fleet, 1: flagged fleets (gated on hb_flag)
    int k1dp;                      // register sweep: 1 = every k = 1 / W = M instance by k1_dp (test path)
    int mmax, r1max, tab, tab_kc;  // table slice shape (kTables)
    unsigned char *gtab;           // kGlobal: per-wave slices
    int64_t gstride;
    const int64_t *x_off;          // halda_fleet_result.x_off (compact x / c layout) or nullptr
    int32_t ks[64];  // the k list travels in the kernel arguments (no copy)
    int32_t Ws[64];  // W = L / k per k (host integer division)
};

// The per-batch part of a sweep's arguments: the table, the results and the per-fleet hand-back flags
// (a launch's own A.F / A.out / A.fflag, or one batch of a steps launch).
// References, so that a launch's own view reads the kernel arguments where they are (no copy held in
// registers).
struct SweepBatch {
    const halda_fleets &F;
    const FleetOut &out;
    uint8_t *fflag;
};

__device__ inline SweepBatch batch_of(const SweepArgs &A) { return SweepBatch{A.F, A.out, A.fflag}; }

// Element offset of instance inst's x / c: the dense layout, or the caller's compact x_off (-1: not
// written).
__device__ inline int64_t xc_at(const SweepArgs &A, int64_t inst) {
    return A.x_off ? A.x_off[inst] : inst * A.xstride;
}

// x / c of one (fleet, k) solution (col layout [w|n|s1|s2|s3|t|z|C] with the fleet's M), written
// by the lane of each device when the caller asked for them.
__device__ inline void put_xc(const SweepArgs &A, const FleetOut &O, int64_t inst, int M, int i, int wl, int n,
                              const int s[4], double z, const FieldRec &r) {
    if (!(A.outs & kOutXC)) return;
    const int64_t at = xc_at(A, inst);
    if (at < 0) return;
    const Dev d = r.dev();
    if (A.outs & kOutX) {
        double *x = O.x + at;
        x[i] = double(wl); x[M + i] = double(n);
        x[2 * M + i] = double(s[0]); x[3 * M + i] = double(s[1]); x[4 * M + i] = double(s[2]);
        x[5 * M + i] = double(s[3]); x[6 * M + i] = z;
    }
    if (A.outs & kOutC) {
        double *c = O.c + at;
        c[i] = d.cw; c[M + i] = d.cn; c[2 * M + i] = d.cs0; c[3 * M + i] = d.cs1; c[4 * M + i] = d.cs2;
        c[5 * M + i] = d.cs3; c[6 * M + i] = 0.0;
    }
}

#ifndef HALDA_SWEEP_TABLE_K1
#define HALDA_SWEEP_TABLE_K1 1  // table launches also run the k = 1 register greedy (else k = 1 via tables)
#endif

__device__ inline void flag_fleet(const SweepArgs &A, uint8_t *fflag, int f, int lane) {
    // the scratch-free register launch (fflag == nullptr) never flags: sweep_fleets runs it alone only
    // when nothing in the batch can need the table launch (no k > 1 with W >= M, R + 1 <= kDpLanes)
    if (lane == 0 && fflag) {
        fflag[f] = 1;
        __hip_atomic_store(A.hb_flag, A.launch_id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
__device__ inline void flag_fleet(const SweepArgs &A, int f, int lane) { flag_fleet(A, A.fflag, f, lane); }

// SG = Wave: one fleet per wave; SG = Seg<16>: one fleet (M <= 16, n_k <= 16) per 16-lane segment,
// tables in the segment's LDS slice, k = 1 register greedy and k > 1 incremental threshold scan
// only: what that cannot do (fast-path fallbacks, non-convex / non-monotone leaves) is flagged for
// the one-fleet-per-wave table launch, as the register-only launch does.
// A fleet handed to sweep_fleet with its fields already loaded (the steps kernel, the resident wave): the
// fields of the lane's device, the fleet's first device, and the lane's k_j / W_j.
struct SweepPre {
    DevFields mf;
    int64_t d0;
    int kj, Wj;
};

// F / O: the batch's table and results (the kernel arguments' A.F / A.out, or one batch of a steps
// launch); kPre: the fleet's fields come prefetched in *pre (every fleet has A.uM <= kK1MaxM devices);
// kXC = false: the x / c outputs are compiled out (the caller guarantees outs has none); kLds: A is in
// LDS (the resident wave), its uniform fields arrive in vector registers.
template <bool kTables, bool kGlobal, class SG = Wave, bool kPre = false, bool kXC = !kPre, bool kLds = false>
__device__ void sweep_fleet(const SweepArgs &A, const halda_fleets &F, const FleetOut &O, int f, const WaveCtx &w,
                            const SG &sg, const SweepPre *pre = nullptr) {
    constexpr int S = SG::S;
    constexpr bool kSeg = S < 64;
    constexpr bool kFirst = !kTables || kSeg;  // a first launch: flags what it leaves to the table launch
    const int lane = sg.sl;  // device index within the fleet
    const SweepModel &Mo = A.Mo;
    HALDA_SSTAMP(0, __builtin_amdgcn_s_memtime());
    HALDA_SSTAMP(7, __builtin_amdgcn_s_memrealtime());
    // lane j: k_j and W_j = L / k_j (kernel arguments; their loads are issued with the fields')
    const bool kl = lane < A.n_k;
    const int kj = kPre ? pre->kj : A.ks[kl ? lane : 0];
    const int Wj = kPre ? pre->Wj : kl ? A.Ws[lane] : 0;
    // the fleet's extent: with one fleet size for the batch, from dev_off[0] read through the scalar
    // cache (the table is read-only to the kernel), so that the field loads are the wave's first
    // vector round trip
    // with one fleet size for the batch the first device is dev_off[0] + f uM; dev_off[0] (0 in the
    // usual table) is read beside the field loads below, not in front of them
    int64_t d0 = kPre ? pre->d0 : A.uM > 0 ? int64_t(f) * A.uM : F.dev_off[f];
    const int M = kPre ? A.uM : A.uM > 0 ? A.uM : int(F.dev_off[f + 1] - d0);
    // the outputs this call writes (a steps launch has no x / c: those paths compile out of it)
    const int outs = kXC ? A.outs : A.outs & (kOutObk | kOutSt);
    bool regs = M <= kK1MaxM;  // lane = device: the k = 1 greedy runs in registers
    if constexpr (kSeg || kPre) regs = true;  // the host sends fleets of at most S / kK1MaxM devices
    FieldRec me = {};
    int bad = 0;
    double tsum = 0.0, xsum = 0.0, kappa = 0.0;
    if (regs) {
        // every field of this lane's device in one round trip (lanes past M read device 0). With one
        // fleet size the loads are issued at once from dev_off[0] = 0 (the usual table) while the
        // scalar read of dev_off[0] is in flight, and reissued only where it is not 0: no dependent
        // round trip in front of the field loads.
        DevFields mf = kPre ? pre->mf : load_fields(F, d0 + (lane < M ? lane : 0));
        if (!kPre && A.uM > 0) {
            // a vector read (returns in order behind the field loads: no wait of its own, unlike a
            // scalar read, whose lgkmcnt wait would also hold the kernel-argument reads)
            const int64_t base = __builtin_amdgcn_readfirstlane(int(F.dev_off[0])) |
                                 (int64_t(__builtin_amdgcn_readfirstlane(int(uint64_t(F.dev_off[0]) >> 32))) << 32);
            if (base != 0) {
                d0 += base;
                mf = load_fields(F, d0 + (lane < M ? lane : 0));
            }
        }
        me = field_rec(Mo, mf, bad);
        bad = lane < M ? bad : 0;
        if (M > 0) fleet_offsets_regs<SG, kLds>(Mo, mf, M, sg, tsum, xsum, kappa);
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
#if defined(HALDA_EXIT_AT) && HALDA_EXIT_AT == 1  // diagnostic: VALU of the records phase alone
    if constexpr (!kTables && !kSeg) {
        const double sink = me.alpha + me.b + me.p_bp + me.p_b + me.cst + double(me.Kset + me.Kvram + me.cls + me.gpu) +
                            tsum + xsum + kappa + double(bad);
        if (lane == 0) O.obj_value[f] = sg.sum_f64(sink);
        return;
    }
#endif
    HALDA_SSTAMP(9, __builtin_amdgcn_s_memrealtime());
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
        if (outs & kOutObk) O.obj_by_k[inst] = kInf;
        if (outs & kOutSt) O.status[inst] = stj;
    }
    if ((outs & kOutXZ) && (outs & kOutXC)) {  // x / c of a settled instance are zero
        uint64_t settled = sg.bits(kl && stj != kOpen);
        const int N = 7 * M + 1;
        while (settled) {
            const int j = __builtin_ctzll(settled);
            settled &= settled - 1;
            const int64_t at = xc_at(A, int64_t(f) * A.n_k + j);
            if (at >= 0)
                for (int cc = lane; cc < N; cc += S) {
                    if (outs & kOutX) O.x[at + cc] = 0.0;
                    if (outs & kOutC) O.c[at + cc] = 0.0;
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
        if constexpr (!kSeg && !kLds) asm volatile("" : "+s"(M));
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
#if defined(HALDA_EXIT_AT) && HALDA_EXIT_AT == 2  // diagnostic: records + the bookkeeping before the greedy
            if constexpr (!kTables && !kSeg) {
                const double sink = me.alpha + me.b + me.p_bp + me.p_b + me.cst + double(me.Kset + me.Kvram + me.cls +
                                    me.gpu + me.W + k + W) + tsum + xsum + kappa;
                if (lane == 0) O.obj_value[f] = sg.sum_f64(sink);
                return;
            }
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
#if defined(HALDA_EXIT_AT) && HALDA_EXIT_AT == 3  // diagnostic: ... + the k = 1 greedy
            if constexpr (!kTables && !kSeg) {
                const double sink = gE + double(e + nE + rounds + rc) + tsum + xsum + kappa;
                if (lane == 0) O.obj_value[f] = sg.sum_f64(sink);
                return;
            }
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
                const bool need_h = kc != 0.0 || (outs & kOutX);
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
                    if (outs & kOutXC) put_xc(A, O, inst, M, lane, wl, n, sl, z, me);
                    if (improved) {
                        O.w[d0 + lane] = wl;
                        O.n[d0 + lane] = n;
                    }
                }
                if (lane == 0 && (outs & kOutXC)) {
                    const int64_t at = xc_at(A, inst);
                    if (at >= 0 && (outs & kOutX)) O.x[at + 7 * M] = hmax;
                    if (at >= 0 && (outs & kOutC)) O.c[at + 7 * M] = kc;
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
                const FieldSrc src{&A.Mo, &F, regs ? &me : nullptr, d0, W, sg.base};
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
                            if (outs & kOutXC) put_xc(A, O, inst, M, i, wl, n, sl, Q > P ? 0.5 * (Q - P) : 0.0, d);
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
                                O.w[d0 + i] = wl;
                                O.n[d0 + i] = n;
                            }
                        }
                    if (lane == 0 && (outs & kOutXC)) {
                        const int64_t at = xc_at(A, inst);
                        if (at >= 0 && (outs & kOutX)) O.x[at + 7 * M] = hmax;
                        if (at >= 0 && (outs & kOutC)) O.c[at + 7 * M] = kc;
                    }
                    HALDA_TSTAMP(8);
                }
                wave_sync();  // tables / st0 are rewritten by the next k
            }
        }
        if (st == HALDA_STATUS_OPTIMAL && M == 0) {
            obj = 0.0;  // c.x = 0; no devices: the offsets are empty sums and kappa is undefined
            improved = obj < best;
            if (lane == 0 && (outs & kOutXC)) {
                const int64_t at = xc_at(A, inst);
                if (at >= 0 && (outs & kOutX)) O.x[at] = 0.0;
                if (at >= 0 && (outs & kOutC)) O.c[at] = kc;
            }
        }
        if (improved) {
            best = obj;
            best_k = k;
        }
        if ((outs & kOutXZ) && st != HALDA_STATUS_OPTIMAL) {  // x / c of a non-optimal instance are zero
            const int N = 7 * M + 1;
            const int64_t at = xc_at(A, inst);
            if (at >= 0)
                for (int cc = lane; cc < N; cc += S) {
                    if (outs & kOutX) O.x[at + cc] = 0.0;
                    if (outs & kOutC) O.c[at + cc] = 0.0;
                }
        }
        if (lane == 0) {
            if (outs & kOutObk) O.obj_by_k[inst] = st == HALDA_STATUS_OPTIMAL ? obj : kInf;
            if (outs & kOutSt) O.status[inst] = st;
        }
    }
    HALDA_SSTAMP(5, __builtin_amdgcn_s_memtime());
    if (lane == 0) {
        O.best_k[f] = best_k;
        O.obj_value[f] = best;
        if (kFirst && A.fflag) A.fflag[f] = 0;
    }
    if (best_k == 0)
        for (int i = lane; i < M; i += S) {
            O.w[d0 + i] = 0;
            O.n[d0 + i] = 0;
        }
    HALDA_SSTAMP(6, __builtin_amdgcn_s_memtime());
    HALDA_SSTAMP(8, __builtin_amdgcn_s_memrealtime());
}

template <bool kTables, bool kGlobal>
__device__ inline void sweep_body(const SweepArgs &A, const SweepBatch &B, unsigned char *slice_base) {
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
    const int nf = B.F.n_fleets;
    for (int64_t b = blockIdx.x; b < nf; b += int64_t(64) * S) {
        const int64_t mine = b + int64_t(lane) * S;
        uint64_t todo = __ballot(mine < nf && (A.want == 0 || B.fflag[mine] == 1));
        while (todo) {
            const int bit = __builtin_ctzll(todo);
            todo &= todo - 1;
            sweep_fleet<kTables, kGlobal>(A, B.F, B.out, int(b + int64_t(bit) * S), w, Wave(lane));
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
    __shared__ uint8_t dparg[kSweepWavesPerBlock][64 * kDpLanes];
    WaveCtx w = {};
    w.dparg = dparg[threadIdx.x >> 6];
    sweep_fleet<false, false>(A, A.F, A.out, f, w, Wave(int(threadIdx.x & 63)));
}

// ---------------------------------------------------------------- steps launch
// halda_sweep_steps_kernel: `steps` consecutive batches of register sweeps (halda_fleets_group_launch)
// in ONE launch. Batch t is group entry (first + t) mod n_desc: its own resident table and result
// arrays, so every batch's outputs are those its own halda_sweep_kernel launch writes (the same
// sweep_fleet code on the same fields). The waves stay resident, six per SIMD (78 VGPRs): the items
// (batch t, fleet f) are taken in batch order, wave g takes items g, g + n_waves, ..., so at any time
// the resident waves work on one or two consecutive batches (neighbouring table rows in HBM) and a
// wave waiting for its next fleet's fields leaves the SIMD to the five others. No per-batch fill
// (every wave of a launch loading at once, then every wave computing) and no launch per batch.
// Measured against the alternatives: register prefetch of the next item's fields
// (116 VGPRs, four waves per SIMD), fleet-order items, staggered wave starts -- all slower.
// A (batch, fleet) item that recurs (more batches than group entries) may be solved by two waves at
// once: they compute the same values and every location's last write is the final value, so the
// results are those of consecutive launches. Every batch shares the shape of the first (n_fleets,
// uM <= kK1MaxM devices, the model, the k list, no x / c outputs): the host checks it.
struct StepsDesc {
    halda_fleets F;
    FleetOut out;
    int64_t base;  // dev_off[0] of the batch's table (read once by the host)
};

struct StepsArgs {
    const StepsDesc *desc;
    int n_desc;
    int first;      // (first item's batch) mod n_desc
    int steps;
    uint8_t *fflag;  // k-slot steps: per (group entry, fleet) hand-back flags, n_desc x n_fleets
};

__device__ inline const __attribute__((address_space(4))) StepsDesc &steps_desc(const StepsArgs &G, int b) {
    return reinterpret_cast<const __attribute__((address_space(4))) StepsDesc *>(uintptr_t(G.desc))[b];
}

__device__ inline halda_fleets steps_fleets(const __attribute__((address_space(4))) StepsDesc &d) {
    halda_fleets F;
    F.n_fleets = d.F.n_fleets; F.min_devices = d.F.min_devices; F.max_devices = d.F.max_devices;
    F.dev_off = d.F.dev_off; F.os_class = d.F.os_class; F.flags = d.F.flags;
    F.scpu_b1 = d.F.scpu_b1; F.sgpu_b1 = d.F.sgpu_b1; F.T_cpu = d.F.T_cpu; F.T_gpu = d.F.T_gpu;
    F.t_kvcpy_cpu = d.F.t_kvcpy_cpu; F.t_kvcpy_gpu = d.F.t_kvcpy_gpu; F.t_ram2vram = d.F.t_ram2vram;
    F.t_vram2ram = d.F.t_vram2ram; F.t_comm = d.F.t_comm; F.s_disk = d.F.s_disk;
    F.d_avail_ram = d.F.d_avail_ram; F.c_cpu = d.F.c_cpu; F.c_gpu = d.F.c_gpu; F.d_avail_cuda = d.F.d_avail_cuda;
    F.d_avail_metal = d.F.d_avail_metal; F.swap = d.F.swap;
    return F;
}

__device__ inline FleetOut steps_out(const __attribute__((address_space(4))) StepsDesc &d) {
    FleetOut o;
    o.best_k = d.out.best_k; o.obj_value = d.out.obj_value; o.w = d.out.w; o.n = d.out.n;
    o.obj_by_k = d.out.obj_by_k; o.status = d.out.status; o.x = d.out.x; o.c = d.out.c;
    return o;
}

// halda_sweep_steps_kernel: the group launch's register form -- `steps` batches of register sweeps in ONE
// launch, one wave per (batch, fleet) item (grid = fleet blocks x steps, blockIdx.y the batch). The
// hardware dispatcher starts each next item's wave on whichever SIMD a wave just left, so one batch's
// tail overlaps the next batch's start, and a wave holds no loop state: 67 VGPRs, seven waves per SIMD
// (the resident-wave form with an item loop: 79 VGPRs, six per SIMD, 49 SGPR spills, 12 % slower).
// Every item runs the same sweep_fleet as halda_sweep_kernel on the same fields (kPre: the fields handed
// in; kXC = false: no x / c), so each batch's results are bit-identical to its own launch.
#ifndef HALDA_STEPS_WAVES
#define HALDA_STEPS_WAVES 6  // occupancy floor of the steps kernel (it takes seven at 67 VGPRs)
#endif

__global__ __launch_bounds__(64 * kSweepWavesPerBlock, HALDA_STEPS_WAVES) void halda_sweep_steps_kernel(SweepArgs A,
                                                                                                   StepsArgs G) {
    const int f = __builtin_amdgcn_readfirstlane(int(blockIdx.x) * kSweepWavesPerBlock + int(threadIdx.x >> 6));
    const int lane = int(threadIdx.x & 63);
    const int nf = A.F.n_fleets, M = A.uM;
    if (f >= nf) return;
    // 32-bit: first < n_desc and blockIdx.y < 65,536 (a 64-bit modulo is ~100 scalar instructions per wave)
    const int b = int((unsigned(G.first) + blockIdx.y) % unsigned(G.n_desc));
    __shared__ uint8_t dparg[kSweepWavesPerBlock][64 * kDpLanes];
    WaveCtx w = {};
    w.dparg = dparg[threadIdx.x >> 6];
    const Wave wv(lane);
    SweepPre cur;
    const bool kl = lane < A.n_k;
    cur.kj = A.ks[kl ? lane : 0];
    cur.Wj = kl ? A.Ws[lane] : 0;
    cur.d0 = steps_desc(G, b).base + int64_t(f) * M;
    // 32-bit device index: group_check admits tables of at most 2^29 devices here
    cur.mf = load_fields32(steps_fleets(steps_desc(G, b)), uint32_t(cur.d0 + (lane < M ? lane : 0)));
    sweep_fleet<false, false, Wave, true>(A, steps_fleets(steps_desc(G, b)), steps_out(steps_desc(G, b)), f, w, wv,
                                          &cur);
}

// ---------------------------------------------------------------- resident single-fleet solver
// halda_resident_kernel: ONE wave that stays resident between single-fleet calls (halda_solve's
// latency path through halda_solve_fleets_host): the host writes the call's sweep arguments and the
// fleet's table into fine-grained pinned memory and bumps `seq`; the wave, polling `seq` across PCIe,
// copies the arguments into LDS, solves the fleet exactly as the per-call register launch does (the
// same sweep_fleet on the same fields, x / c included) writing into the pinned results, and publishes
// `ack` = seq with a system-scope release. No launch and no completion event per call. It leaves when
// the host sets `stop` or after `idle_ticks` of the 100 MHz real-time clock without a request (every
// wave exits: the host relaunches it on its next call), so it never outlives its process by more
// than that. All its stores are vector stores.
struct ResidentBox {
    uint32_t seq;  // host: request number, written after the request
    uint32_t pad0[15];
    uint32_t ack;  // device: the last request done
    uint32_t pad1[15];
    uint32_t stop;  // host: 1 = leave now
    uint32_t pad2[15];
    SweepArgs req;  // host: the request's sweep arguments (one fleet, a register-only plan)
};

struct ResidentArgs {
    ResidentBox *box;
    uint32_t last;        // the request number already answered
    uint32_t idle_ticks;  // s_memrealtime ticks (100 MHz) without a request before the wave leaves
};

__device__ inline uint32_t sys_load(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(64) void halda_resident_kernel(ResidentArgs R) {
    __shared__ SweepArgs As;
    __shared__ uint8_t dparg[64 * kDpLanes];
    const int lane = int(threadIdx.x);
    WaveCtx w = {};
    w.dparg = dparg;
    const Wave wv(lane);
    uint32_t last = R.last;
    uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (true) {
        const uint32_t stop = sys_load(&R.box->stop);
        const uint32_t seq = sys_load(&R.box->seq);
        if (stop) break;
        if (seq == last) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > R.idle_ticks) break;
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the request and table written before seq
        // the sweep arguments into LDS by vector loads (nothing of the request is read through the
        // scalar cache, which does not see the host's writes)
        constexpr int kWords = int(sizeof(SweepArgs) / 4);
        const uint32_t *src = reinterpret_cast<const uint32_t *>(&R.box->req);
        uint32_t *dst = reinterpret_cast<uint32_t *>(&As);
        for (int i = lane; i < kWords; i += 64) dst[i] = sys_load(src + i);
        __builtin_amdgcn_s_waitcnt(0);
        wave_sync();
        SweepPre pre;
        const bool kl = lane < As.n_k;
        pre.kj = As.ks[kl ? lane : 0];
        pre.Wj = kl ? As.Ws[lane] : 0;
        pre.d0 = 0;
        const int M = As.uM;
        pre.mf = load_fields(As.F, lane < M ? lane : 0);
        sweep_fleet<false, false, Wave, true, true, true>(As, As.F, As.out, 0, w, wv, &pre);
        // every result store before ack (system-scope release: the host reads them after it)
        if (lane == 0) __hip_atomic_store(&R.box->ack, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        last = seq;
        t0 = __builtin_amdgcn_s_memrealtime();
        wave_sync();
    }
}

__global__ __launch_bounds__(64, HALDA_SOLVE_WAVES_PER_SIMD) void halda_sweep_tables_kernel(SweepArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    sweep_body<true, false>(A, batch_of(A), smem);
}

__global__ __launch_bounds__(64, HALDA_SOLVE_WAVES_PER_SIMD) void halda_sweep_big_kernel(SweepArgs A) {
    sweep_body<true, true>(A, batch_of(A), A.gtab + int64_t(blockIdx.x) * A.gstride);
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
        if (f < nf) sweep_fleet<true, false, Seg<kSegLanes>>(A, A.F, A.out, int(f), w, sg);
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

struct SlotPick {  // one (segment, k-slot) result in the workgroup's pick area (written after the last use of the
    double obj;    // tables, over them); the slot's (w, n) stay in its wave's registers, and the winning wave
    int st;        // writes them (kslot_pick). st: HALDA_STATUS_* or kSlotFlagged
    int pad;
};

// LDS bytes of one segment's slice of a k-slot (none for a slot without tables: the k = 1 greedy and the
// forced W = M split run in registers).
__host__ __device__ inline int64_t kslot_slice_bytes(int mmax, int tab) {
    return tab > 0 ? seg_slice_bytes(mmax, tab) : 0;
}

struct SlotArgs {
    int n_slot;
    int pick_off;              // LDS byte offset of the pick area (SlotPick [4][n_slot]; over the tables, dead by then)
    int j[kMaxSlots];          // k index of slot q (ascending)
    int tab[kMaxSlots];        // doubles of G (and of H) per segment: max_devices * odd_stride(R + 1), 0: no tables
    int r1[kMaxSlots];         // largest R + 1 of slot q over the batch
    int off[kMaxSlots];        // LDS byte offset of slot q's four segment slices
    int helper;                // slot whose threshold scan is split over n_parts waves (-1: none)
    int n_parts;               // 2 (split) or 0
    int part_wave[kMaxSplitParts - 1];  // the wave that takes part 2 first: a light slot's, or n_slot
    int split_off;             // LDS byte offset of the split areas (SplitArea [4])
    int rec_off;               // LDS byte offset of the workgroup's device records (KslotRecs; over the tables,
                               // which are written only after every wave has read its records)
    int check_wave;            // the wave that checks the split slot's leaves after its own slot (-1: none)
    int opt;                   // 1: an optimistic part 1 where its rows allow (0: the sequential order, a test path)
    int crit_w4;               // table share of the critical slot's wave, in quarters of the others'
    int cut8;                  // the split scan's cut: rank cut8 / 8 of the way up (ScanSplit::cut8)
};
static_assert(kSegLanes == 16, "SplitArea holds 16 lanes per segment");

// Waves of a k-slot workgroup: one per slot, plus an extra helper wave when no other slot can host one.
__host__ __device__ inline int kslot_waves(const SlotArgs &SA) {
    return SA.n_slot + (SA.helper >= 0 && SA.part_wave[0] == SA.n_slot ? 1 : 0);
}

// Part (2 or 3) of the split scan this wave takes first, 0: none.
__device__ inline int kslot_part_of(const SlotArgs &SA, int q) {
    if (SA.helper < 0) return 0;
    for (int h = 0; h < SA.n_parts - 1; ++h)
        if (SA.part_wave[h] == q) return h + 2;
    return 0;
}

// One (fleet, k_j) on a 16-lane segment; the result goes to *pk (segment lane 0 writes obj / st, lane i
// its w / n candidate).
// One fleet of a k-slot workgroup, in registers: its extent, this lane's device record and the
// objective constants (every wave of the workgroup builds the same, from one round of field loads).
struct KslotFleet {
    int64_t d0;
    int M;
    FieldRec me;
    double tsum, xsum, kappa;
    bool anybad;
};

// The workgroup's device records in LDS: wave 0 forms them (kslot_records) and every other wave of
// the workgroup reads them, instead of each wave loading the fields and forming the same records again
// (they are the same four fleets for every slot wave).
struct KslotRecs {
    double alpha[64], b[64], p_bp[64], p_b[64], cst[64];
    int Kset[64], Kvram[64], cg[64];  // cg: cls | gpu << 4
    double tsum[64 / kSegLanes], kappa[64 / kSegLanes];
    int anybad[64 / kSegLanes];
};

__device__ inline void kslot_put_records(KslotRecs *R, const KslotFleet &fd, int lane, int seg) {
    R->alpha[lane] = fd.me.alpha; R->b[lane] = fd.me.b; R->p_bp[lane] = fd.me.p_bp; R->p_b[lane] = fd.me.p_b;
    R->cst[lane] = fd.me.cst;
    R->Kset[lane] = fd.me.Kset; R->Kvram[lane] = fd.me.Kvram; R->cg[lane] = fd.me.cls | (fd.me.gpu << 4);
    if (lane % kSegLanes == 0) {
        R->tsum[seg] = fd.tsum;
        R->kappa[seg] = fd.kappa;
        R->anybad[seg] = fd.anybad ? 1 : 0;
    }
}

__device__ inline KslotFleet kslot_get_records(const SweepArgs &A, const halda_fleets &F, const KslotRecs *R, int f,
                                               int lane, int seg) {
    KslotFleet fd;
    fd.d0 = A.uM > 0 ? int64_t(f) * A.uM + F.dev_off[0] : F.dev_off[f];
    fd.M = A.uM > 0 ? A.uM : int(F.dev_off[f + 1] - fd.d0);
    fd.me.alpha = R->alpha[lane]; fd.me.b = R->b[lane]; fd.me.p_bp = R->p_bp[lane]; fd.me.p_b = R->p_b[lane];
    fd.me.cst = R->cst[lane];
    fd.me.Kset = R->Kset[lane]; fd.me.Kvram = R->Kvram[lane];
    const int cg = R->cg[lane];
    fd.me.cls = cg & 15;
    fd.me.gpu = cg >> 4;
    fd.me.W = 0;
    fd.tsum = R->tsum[seg];
    fd.xsum = 0.0;  // fleet_offsets_regs carries every per-device constant in tsum
    fd.kappa = R->kappa[seg];
    fd.anybad = R->anybad[seg] != 0;
    return fd;
}

__device__ inline KslotFleet kslot_records(const SweepArgs &A, const halda_fleets &F, int f, const Seg<kSegLanes> &sg) {
    KslotFleet fd;
    const int lane = sg.sl;
    fd.d0 = A.uM > 0 ? int64_t(f) * A.uM + F.dev_off[0] : F.dev_off[f];
    fd.M = A.uM > 0 ? A.uM : int(F.dev_off[f + 1] - fd.d0);
    const DevFields mf = load_fields(F, fd.d0 + (lane < fd.M ? lane : 0));
    int bad = 0;
    fd.me = field_rec(A.Mo, mf, bad);
    bad = lane < fd.M ? bad : 0;
    fleet_offsets_regs(A.Mo, mf, fd.M, sg, fd.tsum, fd.xsum, fd.kappa);
    fd.anybad = sg.any(bad != 0);
    return fd;
}

// The (fleet, k_j) instance solves through the tables + threshold scan (not the register greedy /
// forced split, not flagged): the same conditions sweep_kslot's branches test.
__device__ inline bool kslot_uses_tables(const KslotFleet &fd, int k, int W, int r1cap, int tabcap, int mmax) {
    if (!(W < 1000000) || fd.M > W || fd.anybad || k == 1 || W == fd.M || fd.M < 2) return false;
    const int R1 = W - fd.M + 1;
    return fd.M <= mmax && R1 <= r1cap && int64_t(fd.M) * odd_stride(R1) <= tabcap;
}

// Slot p's LDS slice of this segment.
__device__ inline WaveCtx kslot_ctx(const SweepArgs &A, const SlotArgs &SA, int p, unsigned char *smem, int seg) {
    const int tab = SA.tab[p];
    const int64_t tb = align16(int64_t(tab) * 8);
    unsigned char *base = smem + SA.off[p] + int64_t(seg) * kslot_slice_bytes(A.mmax, tab);
    WaveCtx w = {};
    w.G = reinterpret_cast<double *>(base);
    w.H = reinterpret_cast<double *>(base + tb);
    w.st0 = reinterpret_cast<int *>(base + 2 * tb);
    return w;
}

// Phase B of the k-slot workgroup: every wave builds an equal share of ALL the slots' k > 1 tables
// (the (slot, entry) pairs in slot order, cut into one contiguous stretch per wave; lane = device; each
// stretch starts with a full split search, the same least minimisers as one chain, so the same
// tables), instead of each k > 1 wave building its own while the W = M / k = 1 waves idle at the
// barrier: the longest wave's dependent chain loses its table pass.
__device__ void kslot_tables(const SweepArgs &A, const SlotArgs &SA, int q, int crit, const KslotFleet &fd,
                             const Seg<kSegLanes> &sg, unsigned char *smem, int seg) {
    const int lane = sg.sl;
    int total = 0;
    for (int p = 0; p < SA.n_slot; ++p) total += SA.tab[p] > 0 ? SA.r1[p] : 0;
    const int nw = kslot_waves(SA);
    // wave weights in quarters: 4 each, crit_w4 for the critical slot's wave (issue priority: it
    // builds faster and would otherwise wait at the barrier)
    const int cw = crit >= 0 ? SA.crit_w4 : 4;
    const int64_t wt = 4 * int64_t(nw) + cw - 4;
    auto before = [&](int r) { return 4 * int64_t(r) + (crit >= 0 && crit < r ? cw - 4 : 0); };
    const int lo = int(total * before(q) / wt), hi = int(total * before(q + 1) / wt);
    int base = 0;
    for (int p = 0; p < SA.n_slot; ++p) {
        if (SA.tab[p] <= 0) continue;
        const int b0 = base;
        base += SA.r1[p];
        const int a = max(lo, b0) - b0, b = min(hi, base) - b0;
        if (a >= b) continue;
        const int k = A.ks[SA.j[p]], W = A.Ws[SA.j[p]];
        if (!kslot_uses_tables(fd, k, W, SA.r1[p], SA.tab[p], A.mmax)) continue;
        Inst I = {};
        I.M = fd.M;
        I.W = W;
        I.Wd = double(W);
        I.kc = double(k - 1);
        I.iC = 7 * fd.M;
        I.R1 = W - fd.M + 1;
        I.RS = odd_stride(I.R1);
        const WaveCtx w = kslot_ctx(A, SA, p, smem, seg);
        FieldRec rec = fd.me;
        rec.W = W;
        if (lane < fd.M) {
            int n = 0;
            bool have = false;
            for (int e = a; e < min(b, I.R1); ++e) table_entry(rec, w, I, lane, e, n, have);
        }
    }
}

__device__ void sweep_kslot(const SweepArgs &A, const SweepBatch &B, const KslotFleet &fd, int f, int j, int r1cap,
                            int tabcap, const WaveCtx &w, const Seg<kSegLanes> &sg, SlotPick &pk,
                            unsigned long long *t_rec, const ScanSplit sp, int &wl, int &nl) {
    using SG = Seg<kSegLanes>;
    constexpr int S = SG::S;
    const int lane = sg.sl;
    const int M = fd.M;
    FieldRec me = fd.me;
    const double tsum = fd.tsum, xsum = fd.xsum, kappa = fd.kappa;
    const bool anybad = fd.anybad;
#ifndef HALDA_STAMPS
    (void)t_rec;
#endif
    const int k = A.ks[j], W = A.Ws[j];
    const int64_t inst = int64_t(f) * A.n_k + j;
    const double kc = double(k - 1);
    int st;
    double obj = kInf;
    wl = 0;  // this lane's (w, n) in the solution
    nl = 0;
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
                const bool need_h = kc != 0.0 || (A.outs & kOutX);
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
                if (lane < M) put_xc(A, B.out, inst, M, lane, wl, n, sl, z, me);
                if (lane == 0 && (A.outs & kOutXC)) {
                    const int64_t at = xc_at(A, inst);
                    if (at >= 0 && (A.outs & kOutX)) B.out.x[at + 7 * M] = hmax;
                    if (at >= 0 && (A.outs & kOutC)) B.out.c[at + 7 * M] = kc;
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
                // the tables were built by the whole workgroup (kslot_tables, before the barrier)
                int64_t nodes = 0;
                const int feas = dp_pass_lanes(w, I, sg, nodes, t_rec + 4, sp);
#ifdef HALDA_STAMPS
                t_rec[2] = __builtin_amdgcn_s_memtime();
                t_rec[3] = (unsigned long long)nodes;
#endif
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
                        put_xc(A, B.out, inst, M, lane, wl, n, sl, Q > P ? 0.5 * (Q - P) : 0.0, me);
                    }
                    hmax = sg.max_f64(fmax(0.0, hmax));
                    obj = sg.sum_f64(0.0 + g) + kc * hmax;  // the segment kernel's sum (0.0 + g per lane)
                    obj = obj + tsum;
                    obj = obj + xsum;
                    obj = obj + kappa;
                    st = HALDA_STATUS_OPTIMAL;
                    nl = n;
                    if (lane == 0 && (A.outs & kOutXC)) {
                        const int64_t at = xc_at(A, inst);
                        if (at >= 0 && (A.outs & kOutX)) B.out.x[at + 7 * M] = hmax;
                        if (at >= 0 && (A.outs & kOutC)) B.out.c[at + 7 * M] = kc;
                    }
                }
            }
        }
    }
    if (st == kSlotFlagged) {
        flag_fleet(A, B.fflag, f, lane);
    } else {
        if (lane == 0) {
            if (A.outs & kOutObk) B.out.obj_by_k[inst] = st == HALDA_STATUS_OPTIMAL ? obj : kInf;
            if (A.outs & kOutSt) B.out.status[inst] = st;
        }
        if ((A.outs & kOutXZ) && st != HALDA_STATUS_OPTIMAL && (A.outs & kOutXC)) {  // x / c of a non-optimal instance
            const int64_t at = xc_at(A, inst);
            if (at >= 0)
                for (int cc = lane; cc < 7 * M + 1; cc += S) {
                    if (A.outs & kOutX) B.out.x[at + cc] = 0.0;
                    if (A.outs & kOutC) B.out.c[at + cc] = 0.0;
                }
        }
    }
    pk.obj = st == HALDA_STATUS_OPTIMAL ? obj : kInf;  // (lane 0's are the segment's)
    pk.st = st;
}

// The pick of one fleet (segment lanes), run by every slot wave q after the last barrier: best k over the
// slots in ascending k with strict "<"; the winning slot's wave writes its (w, n) from its registers (wl,
// nl), wave 0 the settled k's of no slot, best_k / obj_value, the fleet's flag byte and, when no k is
// feasible, zero (w, n).
__device__ void kslot_pick(const SweepArgs &A, const SweepBatch &B, const SlotArgs &SA, int f, const SlotPick *pk,
                           const Seg<kSegLanes> &sg, int q, int wl, int nl) {
    constexpr int S = kSegLanes;
    const int lane = sg.sl;
    const int64_t d0 = A.uM > 0 ? int64_t(f) * A.uM + B.F.dev_off[0] : B.F.dev_off[f];
    const int M = A.uM > 0 ? A.uM : int(B.F.dev_off[f + 1] - d0);
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
    if (q == bq && lane < M) {
        B.out.w[d0 + lane] = wl;
        B.out.n[d0 + lane] = nl;
    }
    if (q != 0) return;
    // k's of no slot: settled for every fleet of the batch (W >= 1e6 unsupported, else M > W)
    for (int jj = lane; jj < A.n_k; jj += S) {
        bool slot = false;
        for (int q = 0; q < SA.n_slot; ++q) slot = slot || SA.j[q] == jj;
        if (slot) continue;
        const int64_t inst = int64_t(f) * A.n_k + jj;
        const int st = !(A.Ws[jj] < 1000000) ? HALDA_STATUS_UNSUPPORTED : HALDA_STATUS_INFEASIBLE;
        if (A.outs & kOutObk) B.out.obj_by_k[inst] = kInf;
        if (A.outs & kOutSt) B.out.status[inst] = st;
        if ((A.outs & kOutXZ) && (A.outs & kOutXC)) {
            const int64_t at = xc_at(A, inst);
            if (at >= 0)
                for (int cc = 0; cc < 7 * M + 1; ++cc) {
                    if (A.outs & kOutX) B.out.x[at + cc] = 0.0;
                    if (A.outs & kOutC) B.out.c[at + cc] = 0.0;
                }
        }
    }
    if (lane == 0) {
        B.out.best_k[f] = bq >= 0 ? A.ks[SA.j[bq]] : 0;
        B.out.obj_value[f] = best;
        B.fflag[f] = 0;
    }
    if (bq < 0 && lane < M) {
        B.out.w[d0 + lane] = 0;
        B.out.n[d0 + lane] = 0;
    }
}

// The leaf checks of the split slot's rows for an optimistic part 1 (dp_pass_lanes takes rows finite at
// both ends as [0, R1 - 1] without checking them and awaits this verdict before it returns): made by
// SA.check_wave after its own slot, the wave whose slot ends first, while part 1 scans.
__device__ void kslot_check(const SweepArgs &A, const SlotArgs &SA, const KslotFleet &fd, SplitArea *ar,
                            const Seg<kSegLanes> &sg, unsigned char *smem, int seg, bool live) {
    const int p = SA.helper, lane = sg.sl;
    const int j = SA.j[p], k = A.ks[j], W = A.Ws[j];
    if (!SA.opt || !live || !kslot_uses_tables(fd, k, W, SA.r1[p], SA.tab[p], A.mmax)) return;
    const int M = fd.M, R1 = W - M + 1, RS = odd_stride(R1);
    const bool act = lane < M;
    const WaveCtx w = kslot_ctx(A, SA, p, smem, seg);
    const double *G = w.G + int64_t(act ? lane : 0) * RS, *H = w.H + int64_t(act ? lane : 0) * RS;
    if (!leaf_ends_finite(G, R1, act, sg)) return;  // part 1 checks these itself
    int lo = R1, hi = -1, cnt = 0;
    bool ok = true, mono = true;
    leaf_scan(G, H, R1, act, lo, hi, cnt, ok, mono);
    const int v = sg.any(act && (!ok || !mono)) ? 2 : 1;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) __hip_atomic_store(&ar->verdict, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// A helper wave of a k-slot workgroup, after its own slot: its part (T range) of the split slot's
// threshold scan for its segment's fleet, from what part 1 published after its leaf scan and phase-0
// greedy (part 1 publishes on every path: "skip" when it does not scan), into the split area; then
// the flag, on every path (part 1 waits for it only when it scanned). The wait is a wave-uniform
// polling loop in which every segment whose publication is in runs its part at once: a segment must
// never wait behind another one of the same wave (part 1 may publish that one only after its own
// scan, which waits for this segment's flag).
__device__ void kslot_helper(const SweepArgs &A, const SlotArgs &SA, const KslotFleet &fd, SplitArea *ar, int part,
                             const Seg<kSegLanes> &sg, unsigned char *smem, int seg, bool live) {
    const int p = SA.helper, h = part - 2, lane = sg.sl;
    const int j = SA.j[p], k = A.ks[j], W = A.Ws[j];
    // part 1 reaches its leaf scan (else it publishes nothing this wave needs: post at once)
    bool pending = live && kslot_uses_tables(fd, k, W, SA.r1[p], SA.tab[p], A.mmax);
    if (live && lane == 0) ar->alt_best[h] = kInf;
    // an optimistic part 1 (rows finite at both ends: dp_pass_lanes) leaves phase 0 to this wave: the
    // unconstrained allocation into the split slot's st0, then the publication part 1's scan awaits
    if (h == 0 && pending) {
        const int M = fd.M, R1 = W - M + 1, RS = odd_stride(R1);
        const bool act = lane < M;
        const WaveCtx w = kslot_ctx(A, SA, p, smem, seg);
        const double *G = w.G + int64_t(act ? lane : 0) * RS, *H = w.H + int64_t(act ? lane : 0) * RS;
        if (SA.opt && leaf_ends_finite(G, R1, act, sg)) {
            const int hi = act ? R1 - 1 : -1;
            int e = 0;
            phase0_greedy(w.G, RS, R1 - 1, sg, act, hi, e);
            const double s_inf = sg.sum_f64(act ? G[e] : 0.0);
            const double hmax = sg.max_f64(act ? fmax(0.0, H[e]) : 0.0);
            if (act) w.st0[lane] = e;
            split_publish(ar, lane, act, act ? 0 : R1, hi, s_inf, double(k - 1) * hmax + s_inf, 0,
                          sg.sum_i(act ? R1 - 1 : 0));
        }
    }
    while (__ballot(pending)) {
        const int pb = pending ? __hip_atomic_load(&ar->pub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : 0;
        if (pending && pb != 0) {  // segment-uniform
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            if (pb == 1) {
                Inst I = {};
                I.M = fd.M;
                I.W = W;
                I.Wd = double(W);
                I.kc = double(k - 1);
                I.iC = 7 * fd.M;
                I.R1 = W - fd.M + 1;
                I.RS = odd_stride(I.R1);
                const bool act = lane < fd.M;
                LeafInfo li = {};
                li.convex = true;  // part 1 checked every leaf before it published
                li.mono = true;
                li.empty = false;
                li.lo_sum = ar->lo_sum;
                li.cap = ar->capsum;
                li.my_lo = act ? ar->lo[lane] : 0;
                li.my_hi = act ? ar->hi[lane] : -1;
                WaveCtx w = kslot_ctx(A, SA, p, smem, seg);
                w.st0 = ar->alt_e[h];  // this part's result, not the slot's st0
                int64_t nodes = 0;
                ScanSplit sp{part, SA.n_parts, ar};
                sp.cut8 = SA.cut8;
                (void)kc_scan_incremental(w, I, sg, ar->s_inf, ar->best0, nodes, li, sp);
            }
            pending = false;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) __hip_atomic_store(&ar->flag[h], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else if (pending) {
            __builtin_amdgcn_s_sleep(2);
        }
    }
    if (live && !kslot_uses_tables(fd, k, W, SA.r1[p], SA.tab[p], A.mmax)) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) __hip_atomic_store(&ar->flag[h], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

// The slot with the largest k > 1 tables (C2: k = 2): the workgroup's critical path, its threshold scan
// the last thing running; -1 when no slot has tables.
__device__ inline int kslot_crit(const SlotArgs &SA) {
    int crit = -1, r1 = 0;
    for (int p = 0; p < SA.n_slot; ++p)
        if (SA.tab[p] > 0 && SA.r1[p] > r1) {
            r1 = SA.r1[p];
            crit = p;
        }
    return crit;
}

// One k-slot workgroup's four fleets (group g: fleets 4 g .. 4 g + 3 of batch B), every slot wave: the
// records (wave 0, shared through LDS), the tables, each slot's solve and the split scan's parts, the
// pick. Three workgroup barriers on every wave's path.
__device__ void kslot_group(const SweepArgs &A, const SlotArgs &SA, const SweepBatch &B, int64_t g,
                            unsigned char *smem, int crit) {
    constexpr int kPer = 64 / kSegLanes;
    const int lane = threadIdx.x & 63;
    const int q = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));  // this wave's k-slot
    const Seg<kSegLanes> sg(lane);
    const int seg = lane / kSegLanes;
    const int nf = B.F.n_fleets;
    const int64_t f = g * kPer + seg;
    SlotPick *pick = reinterpret_cast<SlotPick *>(smem + SA.pick_off);
    // the critical slot's wave gets the SIMD's issue priority over the other slots' waves (of other
    // workgroups) it shares the SIMD with (its helpers once their own slot is done)
    if (q == crit) __builtin_amdgcn_s_setprio(3);
    else __builtin_amdgcn_s_setprio(0);  // (a helper's raised priority ends with its group)
    SplitArea *split = reinterpret_cast<SplitArea *>(smem + SA.split_off) + seg;
    HALDA_KSTAMPW(0, __builtin_amdgcn_s_memtime());
    // slot 5: the constant-rate clock at start (low 40 bits), the wave's HW_ID[15:0] (SIMD, CU, SE) and
    // XCC_ID[3:0] above
    HALDA_KSTAMPW(5, (__builtin_amdgcn_s_memrealtime() & ((1ull << 40) - 1)) |
                         (uint64_t(__builtin_amdgcn_s_getreg((15 << 11) | 4)) << 40) |
                         (uint64_t(__builtin_amdgcn_s_getreg((3 << 11) | 20)) << 56));
    {
        // the four fleets' device records: formed by wave 0 alone, shared through LDS
        KslotRecs *recs = reinterpret_cast<KslotRecs *>(smem + SA.rec_off);
        KslotFleet fd = {};
        if (q == 0) {
            if (f < nf) {
                fd = kslot_records(A, B.F, int(f), sg);
                kslot_put_records(recs, fd, lane, seg);
            }
        }
        __syncthreads();  // the records are in LDS
        if (q != 0 && f < nf) fd = kslot_get_records(A, B.F, recs, int(f), lane, seg);
        __syncthreads();  // every wave has its records: the tables below may overwrite them
        HALDA_KSTAMPW(1, __builtin_amdgcn_s_memtime());
        if (f < nf) kslot_tables(A, SA, q, crit, fd, sg, smem, seg);
        const int my_part = kslot_part_of(SA, q);
        if (my_part && sg.sl == 0) split->flag[my_part - 2] = 0;  // posted after the barrier
        if (q == SA.helper && sg.sl == 0) {
            split->pub = 0;
            split->verdict = 0;
        }
        HALDA_KSTAMPW(6, __builtin_amdgcn_s_memtime());
        __syncthreads();  // every slot's tables are complete
        HALDA_KSTAMPW(11, __builtin_amdgcn_s_memtime());
        if (q == SA.n_slot) {  // an extra helper wave: no slot of its own
            __builtin_amdgcn_s_setprio(3);
            if (q == SA.check_wave) kslot_check(A, SA, fd, split, sg, smem, seg, f < nf);
            kslot_helper(A, SA, fd, split, my_part, sg, smem, seg, f < nf);
            __syncthreads();  // the pick barriers below
            __syncthreads();
            return;
        }
        const WaveCtx w = kslot_ctx(A, SA, q, smem, seg);
#ifdef HALDA_STAMPS_DUMP  // (-DHALDA_STAMPS -DHALDA_STAMPS_DUMP: tools/kslot_tables.py)
        if (f < kDumpFleets && A.ks[SA.j[q]] == 2 && SA.tab[q] > 0 && lane % kSegLanes < fd.M) {
            const int R1 = A.Ws[SA.j[q]] - fd.M + 1, RS = odd_stride(R1), i = lane % kSegLanes;
            for (int e = 0; e < kDumpE; ++e) {
                const int64_t o = ((int64_t(f) * kDumpDev + i) * kDumpE + e) * 2;
                g_halda_dump[o] = e < R1 ? w.G[i * RS + e] : kInf;
                g_halda_dump[o + 1] = e < R1 ? w.H[i * RS + e] : kInf;
            }
        }
#endif
        unsigned long long t_rec[6] = {0, 0, 0, 0, 0, 0};
        int wl = 0, nl = 0;
        SlotPick mine = {kInf, HALDA_STATUS_INFEASIBLE, 0};
#ifdef HALDA_STAMPS
        ScanSplit sp{q == SA.helper ? 1 : 0, SA.n_parts, split, false, SA.opt != 0,
                     int64_t(blockIdx.x) * SA.n_slot + q < kStampInst
                         ? g_halda_scanprof + (int64_t(blockIdx.x) * SA.n_slot + q) * kScanProf
                         : nullptr};
#else
        ScanSplit sp{q == SA.helper ? 1 : 0, SA.n_parts, split, false, SA.opt != 0};
#endif
        sp.cut8 = SA.cut8;
        if (f < nf)
            sweep_kslot(A, B, fd, int(f), SA.j[q], SA.r1[q], SA.tab[q], w, sg, mine, t_rec, sp, wl, nl);
        if (q == SA.helper && f < nf && sg.sl == 0 && split->pub == 0) split->pub = 2;  // did not scan: helpers skip
        if (q == SA.check_wave) kslot_check(A, SA, fd, split, sg, smem, seg, f < nf);
        if (my_part) {  // after its own slot, at the split slot's priority
            __builtin_amdgcn_s_setprio(3);
            kslot_helper(A, SA, fd, split, my_part, sg, smem, seg, f < nf);
        }
        HALDA_KSTAMPW(7, t_rec[2]);
        HALDA_KSTAMPW(8, t_rec[3]);
        HALDA_KSTAMPW(9, t_rec[4]);
        HALDA_KSTAMPW(10, t_rec[5]);
        HALDA_KSTAMPW(2, __builtin_amdgcn_s_memtime());
        __syncthreads();  // every table read is done: the pick area over them is free
        if (f < nf && sg.sl == 0) pick[seg * SA.n_slot + q] = mine;
        __syncthreads();
        HALDA_KSTAMPW(3, __builtin_amdgcn_s_memtime());
        if (f < nf) kslot_pick(A, B, SA, int(f), pick + seg * SA.n_slot, sg, q, wl, nl);
        HALDA_KSTAMPW(4, __builtin_amdgcn_s_memtime());
    }
}

__global__ __launch_bounds__(64 * kMaxSlots) void halda_sweep_kslot_kernel(SweepArgs A, SlotArgs SA) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    kslot_group(A, SA, batch_of(A), int64_t(blockIdx.x), smem, kslot_crit(SA));
}

// halda_sweep_kslot_steps_kernel: `steps` batches of k-slot sweeps (C2 shapes) in one launch, the group
// launch's k-slot form: one workgroup per item (batch t = blockIdx.y, group of four fleets), so the
// hardware dispatcher hands the next item to whichever CU frees its resources first -- the launch is
// paced by the mean group, not by the slowest of the 1,024 resident at once -- with the per-batch
// kernel's registers (no item loop). Item (t, gg) solves group g = (gg + t * kKslotRot) mod n_groups (a
// bijection per batch), which spreads a slow group's batches over the launch. Fleets a slot flags go to
// the per-batch flag array; halda_sweep_tables_steps_kernel redoes them after the launch.
constexpr int kKslotRot = 389;

__global__ __launch_bounds__(64 * kMaxSlots) void halda_sweep_kslot_steps_kernel(SweepArgs A, SlotArgs SA, StepsArgs G) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nf = A.F.n_fleets;
    const int ng = int(gridDim.x);
    const int t = int(blockIdx.y), gg = int(blockIdx.x);
    // 32-bit: gg < ng, t < 65,536, first < n_desc
    const int g = int((unsigned(gg) + unsigned(t) * unsigned(kKslotRot)) % unsigned(ng));
    const int b = int((unsigned(G.first) + unsigned(t)) % unsigned(G.n_desc));
    kslot_group(A, SA, SweepBatch{steps_fleets(steps_desc(G, b)), steps_out(steps_desc(G, b)), G.fflag + int64_t(b) * nf},
                g, smem, kslot_crit(SA));
}

// The gated table launch behind a k-slot steps launch: blockIdx.y = the group entry (first + y) mod
// n_desc, the fleets its items flagged (gated on the launch's hand-back flag).
__global__ __launch_bounds__(64, HALDA_SOLVE_WAVES_PER_SIMD) void halda_sweep_tables_steps_kernel(SweepArgs A,
                                                                                                StepsArgs G) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int b = int((unsigned(G.first) + blockIdx.y) % unsigned(G.n_desc));
    const halda_fleets F = steps_fleets(steps_desc(G, b));
    const FleetOut O = steps_out(steps_desc(G, b));
    sweep_body<true, false>(A, SweepBatch{F, O, G.fflag + int64_t(b) * A.F.n_fleets}, smem);
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
