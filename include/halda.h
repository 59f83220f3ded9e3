/*
 * halda.h — C ABI of libhalda, the MI355X (gfx950) solver for batches of
 * fixed-k HALDA MILPs.
 *
 * What it replaces. The reference (firstbatchxyz/distilp 0.1.6) solves one
 * fixed-k MILP per (fleet, k) with
 *     res = milp(c=c_obj, integrality=integrality, bounds=bounds,
 *                constraints=constraints, options=options)
 * at src/distilp/solver/halda_p_solver.py:340-346 (scipy 1.15.3 -> HiGHS
 * 1.8.0), and reads only res.success and res.x (:347-353). One call of
 * halda_solve_batch() stands in for a whole batch of such milp() calls: the
 * MILP arrives in CSR form exactly as scipy would hand it to HiGHS
 * (A = [A_ub ; A_eq], the ub rows in the reference's order then the single
 * equality row, scipy/optimize/_milp.py:60-71), and status/x come back per
 * instance with the same meaning as (res.success, res.x).
 *
 * The solve is exact (proven optimum, gap 0): libhalda validates that the CSR
 * has the HALDA structure (columns [w|n|s1|s2|s3|t|z|C], SURVEY.md appendix
 * A) and reduces it to a separable assignment problem that it solves by a
 * min-plus dynamic program over sum(w) on the GPU, with a cycle-time
 * threshold search when k > 1. A matrix without that structure is rejected
 * with HALDA_STATUS_UNSUPPORTED, never approximated.
 *
 * Ownership. Every pointer in halda_batch / halda_result is owned by the
 * caller. halda_solve_batch() takes HOST pointers, copies them to the device
 * and keeps nothing after it returns except grow-only scratch inside ctx.
 * halda_solve_batch_device() takes DEVICE pointers and is asynchronous on the
 * given HIP stream. Calls on one ctx must be serialised (from the host); the
 * work they enqueue on different streams runs concurrently (the per-launch
 * scratch is per stream), so independent batches may alternate over streams to
 * keep several in flight. Use one ctx per GPU.
 * Errors: functions return 0 on success and a negative code otherwise; the
 * message of the last failure on the calling thread is in halda_last_error().
 */
#ifndef HALDA_H
#define HALDA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HALDA_ABI_VERSION 3

/* per-instance status (halda_result.status) */
#define HALDA_STATUS_OPTIMAL 0       /* res.success == True                   */
#define HALDA_STATUS_LIMIT 1         /* reserved (time/node limit)            */
#define HALDA_STATUS_INFEASIBLE 2    /* res.success == False (HiGHS status 2) */
#define HALDA_STATUS_UNSUPPORTED (-1) /* CSR is not a HALDA MILP              */
#define HALDA_STATUS_TOO_LARGE (-2)  /* exceeds the batch's shape summary     */

/* return codes */
#define HALDA_OK 0
#define HALDA_E_ARG (-22)
#define HALDA_E_HIP (-5)
#define HALDA_E_NODEV (-19)

typedef struct halda_batch {
    int32_t n_inst;
    /* Shape summary: upper bounds over the batch that size the on-chip (LDS)
     * scratch. With M = (n_cols-1)/7, W = equality rhs and R = W - sum_i lb(w_i)
     * (the layers left after every device's minimum), per instance:
     *   max_cols   >= n_cols
     *   max_R1     >= R + 1
     *   max_tab    >= M * (R + 1)   over instances with c[C] == 0 (k == 1)
     *   max_tab_kc >= M * (R + 1)   over instances with c[C]  > 0 (k  > 1)
     * halda_solve_batch() (host pointers) computes them itself when all are 0.
     * An instance exceeding them gets HALDA_STATUS_TOO_LARGE. No cap on R + 1 or M
     * beyond the int32 shape fields: instances whose tables exceed the LDS budget
     * are solved on global-memory tables (halda_solve_big_kernel). */
    int32_t max_cols;
    int32_t max_R1;
    int32_t max_tab;
    int32_t max_tab_kc;
    const int32_t *n_cols; /* [n_inst] N = 7M + 1 */
    const int32_t *n_rows; /* [n_inst] ub rows + 1 eq row */
    const int64_t *csr_off; /* [n_inst] start of the instance's row_ptr segment (n_rows + 1 entries) */
    const int64_t *col_off; /* [n_inst] start into c / col_lb / col_ub / integrality / x */
    const int64_t *row_off; /* [n_inst] start into row_lb / row_ub */
    const int32_t *row_ptr; /* absolute offsets into col_idx / val; instances of one fleet may share a segment */
    const int32_t *col_idx;
    const double *val;
    const double *c;
    const double *col_lb;
    const double *col_ub;
    const double *row_lb; /* -inf for ub rows */
    const double *row_ub;
    const uint8_t *integrality;
    double mip_rel_gap; /* accepted for API parity; the solve is exact */
    double mip_abs_gap;
    double time_limit;
    const double *x0; /* optional warm start, may be NULL (unused by the exact solver) */
    const double *y0;
} halda_batch;

typedef struct halda_result {
    int32_t *status;     /* [n_inst] HALDA_STATUS_* */
    double *x;           /* col_off layout, written for OPTIMAL instances */
    double *obj_lin;     /* [n_inst] c.x */
    double *dual_bound;  /* [n_inst] proven lower bound (== obj_lin when OPTIMAL) */
    double *gap;         /* [n_inst] relative gap (0 when OPTIMAL) */
    int64_t *nodes;      /* [n_inst] dynamic-programming passes evaluated */
} halda_result;

/* ABI version (HALDA_ABI_VERSION). */
int halda_version(void);

/* Bind a context to HIP device `device_ordinal` (must be gfx950). */
int halda_init(int device_ordinal, void **ctx);

/* Synchronous solve of a batch given in HOST memory (replaces a loop of milp() calls). */
int halda_solve_batch(void *ctx, const halda_batch *in, halda_result *out);

/* Asynchronous solve of a batch whose arrays are already in DEVICE memory (HBM),
 * enqueued on `stream` (a hipStream_t; NULL = the context's stream). */
int halda_solve_batch_device(void *ctx, const halda_batch *in, halda_result *out, void *stream);

/* halda_solve_batch_device with the caller's settled instances: settled[i] != 0
 * (a DEVICE array of n_inst bytes) states that the caller has already proved
 * instance i bound-infeasible (sum_j ceil(lb(w_j)) > W, e.g. M devices of w >= 1
 * over W = L/k < M layers: the k's milp() returns res.success == False,
 * halda_p_solver.py:369-436). Its result is written as HALDA_STATUS_INFEASIBLE
 * (the screen's own verdict for it: obj_lin = dual_bound = gap = inf, nodes 0)
 * and nothing of it but its flag is read. The batch has no screen launch: its
 * k = 1 kernel (halda_solve_k1_settled_kernel) writes the settled outputs and
 * screens every other instance on the way, with the screen's rules.
 * settled[i] == 0 instances are solved as by halda_solve_batch_device, bit for
 * bit; settled == NULL is halda_solve_batch_device. A settled flag on an
 * instance that is not infeasible is the caller's error (it is not checked). */
int halda_solve_batch_device_settled(void *ctx, const halda_batch *in, halda_result *out, const uint8_t *settled,
                                     void *stream);

/* Device time of the last solve's kernel sequence (both launches) in ms. */
int halda_last_kernel_ms(void *ctx, double *ms);

/* Device time of the last solve's general kernel (halda_solve_kernel) alone, in ms. */
int halda_last_solve_kernel_ms(void *ctx, double *ms);

/* Record the per-launch HIP events the *_ms queries read (on = 1, the default);
 * off drops four event records per launch from the stream. */
int halda_set_timing(void *ctx, int on);

/* Device time of the last solve per launch, in ms: ms3[0] the screen kernel
 * (halda_screen_kernel), ms3[1] the persistent k = 1 kernel (halda_solve_k1_kernel),
 * ms3[2] the general kernel's launches (k > 1, then k = 1 wide / hand-backs). A settled batch
 * (halda_solve_batch_device_settled) has no screen launch: ms3[0] = 0 and ms3[1] is its k = 1 kernel
 * (halda_solve_k1_settled_kernel, which screens on its way). */
int halda_last_phase_ms(void *ctx, double *ms3);

/* ------------------------------------------------------------------------
 * Whole k-sweeps on the GPU: lowering + solve + argmin over k.
 *
 * halda_solve_fleets() runs the reference's `halda_solve` for a batch of
 * fleets (halda_p_solver.py:369-436): per fleet it lowers every k-candidate
 * to the fixed-k MILP exactly as solve_fixed_k_milp does
 * (halda_p_solver.py:59-338 with the coefficients of dense_common.py:25-230,
 * same operation order, bit-identical CSR to the host lowering), solves them
 * with the kernels above and keeps the best k by the reference's rule
 * (ascending k, strict "<" on obj_value). Inputs are a flat table of the
 * device fields the formulas read (one entry per device, fleets contiguous),
 * so a stream of re-profiled fleets never goes through per-device Python
 * objects. obj_value = c.x + sum t_comm + sum xi + kappa is formed on the GPU
 * (c.x summed in a fixed tree order: within 1e-12 relative of NumPy's dot).
 * ------------------------------------------------------------------------ */

typedef struct halda_model {
    double f_q_b1;      /* ModelProfile.f_q["b_1"] (when has_f_q) */
    double f_out_b1;    /* ModelProfile.f_out["b_1"] (when has_f_out) */
    int32_t has_f_q, has_f_out;
    double b_prime;     /* b_prime(model, kv) (dense_common.py:25-46), an integer value */
    double b_layer, b_in, b_out, V;
    int32_t L;
} halda_model;

/* halda_fleets.flags bits, per device */
#define HALDA_DEV_HEAD 1       /* is_head */
#define HALDA_DEV_UMA 2        /* is_unified_mem */
#define HALDA_DEV_CPU_RATE 4   /* Q in scpu: scpu_b1 = scpu[Q]["b_1"] */
#define HALDA_DEV_GPU 8        /* a GPU FLOPs table and load throughput (beta is active) */
#define HALDA_DEV_GPU_RATE 16  /* ... and Q in that table: sgpu_b1 = table[Q]["b_1"] */
#define HALDA_DEV_CUDA_OK 32   /* has_cuda and d_avail_cuda is not None */
#define HALDA_DEV_METAL_OK 64  /* has_metal and d_avail_metal is not None */
#define HALDA_DEV_METAL_AVAIL 128 /* d_avail_metal is not None (M2 RAM row present) */

typedef struct halda_fleets {
    int32_t n_fleets;
    int32_t min_devices, max_devices; /* over the batch (size the scratch and the shape summary) */
    const int64_t *dev_off;           /* [n_fleets + 1]: fleet f owns devices dev_off[f] .. dev_off[f+1]-1 */
    const uint8_t *os_class;          /* 1 mac_no_metal (M1), 2 mac_metal (M2), 3 anything else (M3) */
    const uint8_t *flags;             /* HALDA_DEV_* */
    const double *scpu_b1, *sgpu_b1;  /* FLOP/s for batch 1 at quantization Q */
    const double *T_cpu, *T_gpu;      /* T_gpu: the load throughput matching the GPU table */
    const double *t_kvcpy_cpu, *t_kvcpy_gpu, *t_ram2vram, *t_vram2ram, *t_comm, *s_disk;
    /* byte counts: the profiles' integers as doubles (exact below 2^53 bytes; ABI 3 -- ABI 2 had int64) */
    const double *d_avail_ram, *c_cpu, *c_gpu, *d_avail_cuda, *d_avail_metal;
    const double *swap;               /* min(d_bytes_can_swap, d_swap_avail) for android, else 0 */
} halda_fleets;

typedef struct halda_fleet_result {
    int32_t *best_k;     /* [n_fleets] best k, 0 when no k is feasible */
    double *obj_value;   /* [n_fleets] */
    int32_t *w, *n;      /* [dev_off[n_fleets]] device layout */
    double *obj_by_k;    /* [n_fleets * n_k] obj_value per k (+inf infeasible); may be NULL */
    int32_t *status;     /* [n_fleets * n_k] HALDA_STATUS_* per k; may be NULL */
    double *x;           /* [n_fleets * n_k * (7 max_devices + 1)] x per (fleet, k), column layout; may be NULL */
    double *c;           /* same layout: the lowered objective c per (fleet, k); may be NULL */
    /* Optional compact x / c layout (ABI 2): x_off[f * n_k + j] = element offset of instance (f, k_j)'s
     * 7 M_f + 1 entries in x and c, or -1 for an instance whose x / c are not wanted (e.g. L / k < M_f,
     * which cannot be optimal). NULL: the dense layout above. Device memory for halda_solve_fleets,
     * host memory for halda_solve_fleets_host / _multi (x and c then hold max(x_off + 7 M_f + 1)). */
    const int64_t *x_off;
} halda_fleet_result;

/* Asynchronous on `stream` (NULL = the context's stream): the halda_fleets and
 * halda_fleet_result arrays are device memory; ks (host memory, n_k entries)
 * is ascending, unique, > 0 (at most 64 entries on the fused path). Shape limit:
 * (L / ks[0] - min_devices + 1) * max_devices <= 2^27; tables beyond the LDS budget go to HBM. */
int halda_solve_fleets(void *ctx, const halda_model *model, const halda_fleets *fleets, const int32_t *ks,
                       int32_t n_k, halda_fleet_result *out, void *stream);

/* A prepared halda_solve_fleets for a table that stays resident (a streaming deployment re-solves the
 * same buffers as their contents change): the kernel choice, grids, LDS slices and kernel arguments are
 * derived from the shapes once, at creation, so each halda_fleets_plan_launch() is one or two kernel
 * enqueues on `stream` (NULL = the context's stream), asynchronous, with the results of a
 * halda_solve_fleets call on the same arguments. The device arrays behind `fleets` / `out` must stay
 * allocated with the same shapes (n_fleets, dev_off, min / max devices) while the plan lives; their
 * contents may change between launches. A halda_set_fleets_path on the context re-plans the plan at its
 * next launch. Launches of one context's plans must be serialised on the host, like every call on
 * that context. */
int halda_fleets_plan_create(void *ctx, const halda_model *model, const halda_fleets *fleets, const int32_t *ks,
                             int32_t n_k, const halda_fleet_result *out, void **plan);
int halda_fleets_plan_launch(void *plan, void *stream);
/* `steps` launches in one call, launch t of plans[(first + t) % n_plans] on streams[(first + t) %
 * n_streams] (a streaming caller's batches rotating over resident tables and streams, without a host
 * round trip per batch); stops at the first failing launch and returns its code. */
int halda_fleets_plan_launch_many(void *const *plans, int32_t n_plans, void *const *streams, int32_t n_streams,
                                  int64_t first, int32_t steps);
void halda_fleets_plan_free(void *plan);

/* A group of prepared plans run as a stream of batches: halda_fleets_group_launch(group, first, steps,
 * stream) solves batch t = plans[(first + t) % n_plans] for t = 0 .. steps - 1, each batch's results in
 * its own plan's arrays, exactly as halda_fleets_plan_launch_many(plans, n_plans, &stream, 1, first,
 * steps) would leave them. When every plan is a register sweep of one shape (the same model, k list,
 * fleet count and fleet size uM <= 64, no x / c outputs: C3's resident copies) the steps run as ONE
 * launch of one wave per (batch, fleet) item (steps <= 65,535); when every plan is a k-slot
 * sweep of one shape (fleets of <= 16 devices with k > 1 tables: C2) as one k-slot launch of one
 * workgroup per (batch, group of four fleets) item (steps <= 65,535), then one gated table launch for the
 * fleets they flagged (*persistent = 1); otherwise batch by batch on `stream` (*persistent = 0). The group copies what it
 * needs from the plans at creation (the plans may be freed after it); the tables and result arrays
 * behind them must stay allocated while the group lives. Plans and groups fail with HALDA_E_ARG once
 * their context was freed. Replaces the per-batch loop over halda_solve (halda_p_solver.py:369-436)
 * that a streaming caller runs. */
int halda_fleets_group_create(void *const *plans, int32_t n_plans, void **group, int32_t *persistent);
int halda_fleets_group_launch(void *group, int64_t first, int32_t steps, void *stream);
void halda_fleets_group_free(void *group);

/* How halda_solve_fleets runs (default 1; HALDA_FLEETS_PATH=csr / =wave at halda_init select 0 / 2):
 * 1 the fused sweep (halda_sweep_kernel: every (fleet, k) built in registers from the device
 *   fields, solved and compared in one wave per fleet; no MILP is materialised); batches of more
 *   than 64 fleets of at most 16 devices that need k > 1 tables run four fleets per wave, one per
 *   16-lane segment, and one wave per open k (halda_sweep_kslot_kernel: the best k picked in the
 *   workgroup), or, when its LDS does not fit (and at most 16 k), every k in turn in one wave
 *   (halda_sweep_seg_kernel);
 * 2 the fused sweep, one fleet per wave only;
 * 4 the fused sweep with the segment kernel instead of the k-slot kernel;
 * 5 (test path) the fused sweep with the k-slot kernel's k = 2 threshold scan unsplit (path 1 splits
 *   it over two waves);
 * 6 (test path) the fused sweep with the k-slot kernel's split scan in sequential order (path 1 lets
 *   its part 1 take rows finite at both ends unchecked, the leaf checks and phase 0 made by other waves
 *   of the workgroup; here part 1 makes them itself, as it does for any other row);
 * 0 the CSR pipeline (lowering kernel -> the halda_solve_batch kernels -> pick kernel), which also
 *   keeps the lowered batch for halda_last_lowered. All give the same statuses, x and k.
 * HALDA_E_ARG for any other path. */
int halda_set_fleets_path(void *ctx, int path);

/* Device time of the last halda_solve_fleets call per launch, in ms (per-launch events on, see
 * halda_set_timing; 0 for launches that did not run; ms8 holds 9 entries): ms8[0] the fused sweep kernel
 * (halda_sweep_kernel), ms8[7] the segment kernel (halda_sweep_seg_kernel), ms8[8] the k-slot kernel
 * (halda_sweep_kslot_kernel), ms8[1] their table launch (halda_sweep_tables_kernel / halda_sweep_big_kernel:
 * the flagged fleets, or the whole batch when k > 1 / wide fleets need tables from the start);
 * CSR pipeline: ms8[2] lowering, ms8[3] screen, ms8[4] k = 1 solve, ms8[5] general kernel,
 * ms8[6] pick. */
int halda_last_fleet_ms(void *ctx, double *ms8);

/* Synchronous variant on HOST arrays (halda_fleets / halda_fleet_result in host
 * memory; obj_by_k and status may be NULL). A one-fleet call (a single halda_solve) is answered by a
 * wave the context keeps resident on its own stream: it stays for up to 2 ms after each answer (or
 * until halda_resident_release / halda_free), and any device-wide wait of libhalda's HIP runtime
 * (hipDeviceSynchronize, hipFree) in that window waits for it. */
int halda_solve_fleets_host(void *ctx, const halda_model *model, const halda_fleets *fleets, const int32_t *ks,
                            int32_t n_k, halda_fleet_result *out);

/* Ask the context's resident wave (above) to leave now and wait until it has (a no-op when none
 * runs); the next one-fleet call relaunches it. For callers about to synchronise the whole device. */
int halda_resident_release(void *ctx);

/* Page-locked host memory for halda_solve_fleets_host's arrays. When EVERY array of the call's fleets and
 * results (and x_off) lies in blocks from halda_host_alloc, a call above the zero-copy size copies straight
 * between them and device memory (one DMA per array) instead of staging both ways through the context's
 * own pinned buffer with host memcpys -- the batch API packs its fleet table into such a block
 * (distilp_amd/solver/fleets.py). The results are the same either way. */
int halda_host_alloc(size_t bytes, void **ptr);
void halda_host_free(void *ptr);

/* Several GPUs from one process: a context per device (ordinals may repeat), and
 * halda_solve_fleets_host over all of them -- the fleets are dealt out in contiguous blocks, one host
 * thread per device, results written at each block's offsets. Fleets are independent, so no
 * collective is involved; multi-process / multi-node callers use one halda_init context per rank
 * (distilp_amd/distributed.py: torch.distributed / RCCL around it). */
int halda_init_multi(int n_dev, const int *ordinals, void **mctx);
int halda_solve_fleets_multi(void *mctx, const halda_model *model, const halda_fleets *fleets, const int32_t *ks,
                             int32_t n_k, halda_fleet_result *out);
void halda_free_multi(void *mctx);

/* Latency mode across processes, one per GPU: the ranks of an RCCL communicator
 * (ncclComm_t, passed as void*) each sweep their share of the k-candidates of every fleet --
 * ks[rank], ks[rank + world], ... -- on their own GPU (halda_solve_fleets), then agree on each fleet's
 * best k by the reference's rule (smallest obj_value, ties to the smallest k, halda_p_solver.py:407)
 * with device-side all-reduces over xGMI: MIN of obj_value, MIN of the k reaching it, SUM of the owner's
 * (w, n), and MIN / MAX of obj_by_k / status when those are requested. Every rank ends with the same
 * halda_fleet_result (device arrays; x and c must be NULL). Asynchronous on `stream`; every rank calls
 * it with the same fleets and ks. obj_value is the GPU-formed objective (see halda_solve_fleets).
 * halda_comm_unique_id / halda_comm_init / halda_comm_destroy wrap ncclGetUniqueId / ncclCommInitRank
 * (the 128-byte id goes from one rank to the others by any channel) for callers without their own
 * communicator. */
int halda_comm_unique_id(void *id128);
int halda_comm_init(void **comm, int world, int rank, const void *id128, int device_ordinal);
void halda_comm_destroy(void *comm);
int halda_solve_fleets_sharded(void *ctx, void *comm, const halda_model *model, const halda_fleets *fleets,
                               const int32_t *ks, int32_t n_k, halda_fleet_result *out, void *stream);

/* Latency mode's exact step sequence for `world` virtual ranks (1..16) on ONE device, for tests and
 * measurement where a node's GPUs are not available: every virtual rank's sub-sweep and shard kernels run
 * into its own result arrays (library scratch), and each RCCL all-reduce of halda_solve_fleets_sharded is
 * replaced, in the same order, by one device kernel reducing over the virtual ranks' arrays (MIN / SUM /
 * MAX as there). The arrays of virtual rank `report_rank` are the caller's `out`. Asynchronous on
 * `stream`. */
int halda_solve_fleets_sharded_emulated(void *ctx, int32_t world, int32_t report_rank, const halda_model *model,
                                        const halda_fleets *fleets, const int32_t *ks, int32_t n_k,
                                        halda_fleet_result *out, void *stream);

/* The lowered batch of the last halda_solve_fleets call (device pointers into ctx
 * scratch, valid until the next call on ctx): for tests and diagnostics. An
 * instance with L / k < M (bound-infeasible) carries only its header, w bounds,
 * c[C] and equality-row bounds. x / c of halda_fleet_result are 0 for every
 * instance that is not OPTIMAL. */
int halda_last_lowered(void *ctx, halda_batch *lowered, halda_result *solved);

/* Bytes of dynamic LDS per wave of the general kernel's larger launch for a batch of this shape. */
int64_t halda_lds_bytes(int32_t max_cols, int32_t max_R1, int32_t max_tab, int32_t max_tab_kc);

/* Copy the calling thread's last error message into buf. Returns its length. */
int halda_last_error(char *buf, size_t len);

void halda_free(void *ctx);

#ifdef __cplusplus
}
#endif

#endif /* HALDA_H */
