// libhalda — exact batched solver for fixed-k HALDA MILPs on MI355X (gfx950).
//
// Replaces the per-(fleet, k) call scipy.optimize.milp -> HiGHS made by the
// reference at src/distilp/solver/halda_p_solver.py:340-346 (halda_solve_batch) and
// the whole halda_solve k-sweep of :369-436 (halda_solve_fleets); the C ABI is in
// include/halda.h, the design (and why the solve is exact) in DESIGN.md.
//
// One translation unit in four files:
//   halda_prims.hpp  constants, stamps, LDS slices, wave / segment reductions;
//   halda_solve.hpp  the milp() replacement: records, splits, greedy, DP, CSR decode,
//                    screen / k = 1 / general kernels;
//   halda_sweep.hpp  the k-sweep: GPU lowering, fused sweep kernels, k-slot kernel, pick;
//   halda.hip        host side: contexts, launch sequences, the C ABI, RCCL latency mode.
// Floating point keeps the reference's operation order (-ffp-contract=off).

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "halda.h"

namespace {
// Page-locked host blocks handed out by halda_host_alloc: a call whose every host array lies in one of
// them copies straight between them and device memory (no staging memcpy through the context's buffer).
std::mutex g_host_mu;
std::vector<std::pair<uintptr_t, size_t>> g_host_blocks;

bool in_host_block(const void *p, size_t bytes) {
    if (!p) return true;  // an absent optional array
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    std::lock_guard<std::mutex> lock(g_host_mu);
    for (const auto &b : g_host_blocks)
        if (a >= b.first && a - b.first <= b.second && bytes <= b.second - (a - b.first)) return true;
    return false;
}


#include "halda_prims.hpp"
#include "halda_solve.hpp"
#include "halda_sweep.hpp"

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

struct Ctx;
// A prepared plan or group bound to a context: halda_free detaches every live one (c = nullptr), so a
// launch through it after the context is gone fails with HALDA_E_ARG instead of touching freed memory.
struct CtxHandle {
    Ctx *c = nullptr;
};

struct Ctx {
    int device = 0;
    int cus = 256;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, evs = nullptr, evk = nullptr;  // start, end, after k = 1, after screen
    bool timed = false;
    bool timing = true;  // record the per-launch HIP events (halda_set_timing)
    int *hb_flag = nullptr;  // launch id of the last launch with a k = 1 hand-back
    int launch_id = 0;
    void *scratch = nullptr;  // host-API staging (device)
    void *pinned = nullptr;   // host-API staging (pinned host), one PCIe copy each way
    void *pinned_dev = nullptr;  // its device address (zero-copy small calls), looked up once
    // the resident single-fleet solver (halda_resident_kernel): its mailbox (fine-grained pinned memory),
    // stream, exit event, the last request number, whether a launch of it may still be running
    ResidentBox *rbox = nullptr;
    void *rbox_dev = nullptr;
    hipStream_t rstream = nullptr;
    hipEvent_t rdone = nullptr;
    uint32_t rseq = 0;
    bool rlive = false;
    bool resident = true;  // HALDA_RESIDENT=0 at halda_init: every small call launches its own kernel
    bool resident_drop = false;  // HALDA_RESIDENT_TEST=drop (fault injection): requests are never posted
    std::vector<void *> retired;  // pinned buffers a resident wave that would not stop may still write
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
    int kslot_split = 2;                         // k-slot launch: the longest scan split over 2 waves (0: unsplit)
    bool kslot_opt = true;                       // ... its part 1 optimistic (leaf checks / phase 0 by other waves)
    int kslot_cut8 = 4;                          // k-slot split scan's cut, eighths (HALDA_KSLOT_CUT8, A/B;
                                                 // 4/8 since five workgroups share a CU: 5/8 before)
    int kslot_pad = 0;                           // HALDA_KSLOT_LDS_PAD (diagnostic): unused LDS bytes per
                                                 // k-slot workgroup, to measure the occupancy's effect
    int kslot_crit_w4 = 8;                       // k-slot table share of the critical slot's wave (quarters; 2x:
                                                 // measured best of 7..12 since part 1 leaves its leaf checks and
                                                 // phase 0 to other waves; 2.5x before)
    bool fleet_timed = false;
    bool fleets_fused = true;      // halda_solve_fleets: the fused sweep (default) or the CSR pipeline
    bool seg_sweep = true;         // fused sweep: lane-segment launch for fleets of <= kSegLanes devices
    bool k1_force_dp = false;      // fused sweep, test path: every register-launch k = 1 solve by k1_dp
    bool x_zero = true;            // fused sweep: x / c of non-optimal instances written as zeros
    bool host_copy = false;        // halda_solve_fleets_host: PCIe copies even for small calls (HALDA_HOST_PATH=copy)
    bool fused_screen = true;      // a settled batch screens inside its k = 1 kernel (HALDA_FUSED_SCREEN=0: screen launch)
    bool fused_last = false;       // the last CSR launch screened in its k = 1 kernel (halda_last_phase_ms)
    bool last_fleet_fused = false;
    int path_gen = 0;              // bumped by halda_set_fleets_path: prepared plans re-plan on their next launch
    void *shard = nullptr;         // rank-local results of halda_solve_fleets_sharded
    size_t shard_bytes = 0;
    void *emu = nullptr;           // the other virtual ranks' results of halda_solve_fleets_sharded_emulated
    size_t emu_bytes = 0;
    // The fused sweep's scratch (per-fleet "needs the table launch" bytes, the hand-back flag) per
    // stream: launches on one stream are ordered by it, so batches enqueued on different streams use
    // different slots and need no cross-stream ordering (they overlap on the device). A slot moving to
    // another stream waits for the launches already enqueued on the stream it leaves.
    struct SweepSlot {
        hipStream_t stream = nullptr;
        bool used = false;
        uint64_t tick = 0;
        uint8_t *fflag = nullptr;
        size_t fflag_bytes = 0;
        uint8_t *cls = nullptr;  // the CSR pipeline's per-instance verdict bytes
        size_t cls_bytes = 0;
        int *hb = nullptr;
        hipEvent_t ev = nullptr;
    };
    static constexpr int kSweepSlots = 8;
    SweepSlot sws[kSweepSlots];
    uint64_t sws_tick = 0;
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
    // The dynamic-LDS limit is a per-function attribute of the whole process: it only ever rises here
    // (the largest size any plan of any context asked for), so a plan made for a large slice stays
    // launchable after a smaller one was planned for the same kernel.
    // Keyed by (device, kernel) -- contexts on several devices (halda_init_multi) each raise their own --
    // and guarded by a lock: contexts may be driven from different host threads.
    struct LdsAttr {
        int device;
        const void *fn;
        int64_t lds;
    };
    static constexpr int kLdsAttrs = 64;
    static inline std::mutex lds_mu;
    static inline LdsAttr lds_attr[kLdsAttrs] = {};
    static inline int n_lds_attr = 0;
    static hipError_t ensure_lds(const void *fn, int64_t lds) {
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        std::lock_guard<std::mutex> lock(lds_mu);
        int i = 0;
        while (i < n_lds_attr && !(lds_attr[i].fn == fn && lds_attr[i].device == dev)) ++i;
        if (i < n_lds_attr && lds_attr[i].lds >= lds) return hipSuccess;
        e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
        if (i == n_lds_attr && n_lds_attr < kLdsAttrs) ++n_lds_attr;
        if (i < kLdsAttrs) lds_attr[i] = LdsAttr{dev, fn, lds};
        return hipSuccess;
    }
    // process-unique (a freed context's address may be reused by the next one): keys the plan cache
    static inline std::atomic<uint64_t> next_uid{1};
    uint64_t uid = next_uid.fetch_add(1);
    std::vector<CtxHandle *> handles;  // live plans / groups made on this context
    void detach(CtxHandle *h) { handles.erase(std::remove(handles.begin(), handles.end(), h), handles.end()); }
    hipError_t occupancy(const void *fn, int64_t lds, int *per_cu) {
        hipError_t e = ensure_lds(fn, lds);
        if (e != hipSuccess) return e;
        for (int i = 0; i < n_occ; ++i)
            if (occ[i].fn == fn && occ[i].lds == lds) {
                if (per_cu) *per_cu = occ[i].per_cu;
                return hipSuccess;
            }
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

// A stream's scratch slot (see Ctx::SweepSlot): grown to hold `need` bytes at *buf.
int grow(uint8_t **buf, size_t *bytes, size_t need) {
    need = (need + 255) & ~size_t(255);
    if (need > *bytes) {
        if (*buf) HIP_TRY(hipFree(*buf));  // hipFree waits for the device
        *buf = nullptr;
        *bytes = 0;
        HIP_TRY(hipMalloc(buf, need));
        *bytes = need;
    }
    return HALDA_OK;
}

// The fused sweep's scratch slot for stream s with room for nf fleet flags (see Ctx::SweepSlot).
int sweep_slot(Ctx *c, hipStream_t s, int64_t nf, Ctx::SweepSlot **out) {
    Ctx::SweepSlot *slot = nullptr;
    for (auto &x : c->sws)
        if (x.used && x.stream == s) slot = &x;
    if (!slot) {
        for (auto &x : c->sws)
            if (!slot || (!x.used && slot->used) || (x.used == slot->used && x.tick < slot->tick)) slot = &x;
        if (slot->used) {  // taken over from another stream: after everything enqueued there so far
            HIP_TRY(hipEventRecord(slot->ev, slot->stream));
            HIP_TRY(hipStreamWaitEvent(s, slot->ev, 0));
        } else {
            HIP_TRY(hipEventCreateWithFlags(&slot->ev, hipEventDisableTiming));
            HIP_TRY(hipMalloc(&slot->hb, 256));
            HIP_TRY(hipMemsetAsync(slot->hb, 0, 256, s));
            slot->used = true;
        }
        slot->stream = s;
    }
    slot->tick = ++c->sws_tick;
    if (nf > 0) {
        const int rc = grow(&slot->fflag, &slot->fflag_bytes, size_t(nf));
        if (rc != HALDA_OK) return rc;
    }
    *out = slot;
    return HALDA_OK;
}

int launch(Ctx *ctx, const halda_batch &in, const halda_result &out, hipStream_t stream,
           const uint8_t *settled = nullptr) {
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
    // the verdict bytes and the hand-back flag are this stream's (its scratch slot): launches on other
    // streams need no ordering with this one; only the global tables of the big launch are shared
    Ctx::SweepSlot *slot = nullptr;
    {
        int rc = sweep_slot(ctx, stream, 0, &slot);
        if (rc == HALDA_OK) rc = grow(&slot->cls, &slot->cls_bytes, n);
        if (rc != HALDA_OK) return rc;
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
    if (big) {
        const int rc = order_after_previous(ctx, stream);
        if (rc != HALDA_OK) return rc;
    }
    uint8_t *cls = slot->cls;
    int *hb_flag = slot->hb;
    int *gen_flag = slot->hb + 16;  // its own 64 B of the slot's flag block
    const int launch_id = ++ctx->launch_id;  // tags this launch's flags: k = 1 hand-backs, k > 1 work (no reset)
    if (ctx->timing) HIP_TRY(hipEventRecord(ctx->ev0, stream));
    const int64_t lds1 = make_k1_slice(std::min(mmax, kK1MaxM)).total;
    if (settled && ctx->fused_screen) {
        // a settled batch: no screen launch -- the persistent k = 1 kernel writes the settled instances'
        // outputs and screens every other instance on its way (halda_solve_k1_settled_kernel)
        ctx->fused_last = true;
        int per_cu = 0;
        HIP_TRY(ctx->occupancy(reinterpret_cast<const void *>(halda_solve_k1_settled_kernel), lds1, &per_cu));
        const int grid = int(std::max<int64_t>(1, std::min<int64_t>(int64_t(ctx->cus) * per_cu, in.n_inst)));
        hipLaunchKernelGGL(halda_solve_k1_settled_kernel, dim3(grid), dim3(64), size_t(lds1), stream, in, out, cls,
                           mmax, hb_flag, launch_id, settled, gen_flag, in.max_R1, int(tab), int(tab_kc));
        HIP_TRY(hipGetLastError());
    } else {
        ctx->fused_last = false;
        // screen kernel (8 instances per wave), then a persistent k = 1 kernel
        const int64_t screen_waves = (int64_t(in.n_inst) + kScreenPer - 1) / kScreenPer;
        hipLaunchKernelGGL(halda_screen_kernel, dim3(unsigned((screen_waves + 3) / 4)), dim3(256), 0, stream, in, out,
                           cls, mmax, in.max_R1, int(tab), int(tab_kc), settled, gen_flag, launch_id);
        HIP_TRY(hipGetLastError());
        if (ctx->timing) HIP_TRY(hipEventRecord(ctx->evk, stream));
        int per_cu = 0;
        HIP_TRY(ctx->occupancy(reinterpret_cast<const void *>(halda_solve_k1_kernel), lds1, &per_cu));
        const int grid = int(std::max<int64_t>(1, std::min<int64_t>(int64_t(ctx->cus) * per_cu, in.n_inst)));
        hipLaunchKernelGGL(halda_solve_k1_kernel, dim3(grid), dim3(64), size_t(lds1), stream, in, out, cls, mmax,
                           hb_flag, launch_id);
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
        // gated on the screen's flag: a batch whose k > 1 instances were all settled by the screen (C3:
        // every k > 1 is bound-infeasible) leaves this launch nothing to do
        hipLaunchKernelGGL(halda_solve_kernel, dim3(grid), dim3(64), size_t(lds_kc), stream, in, out, cls, ls.mmax,
                           ls.r1, 0, ls.tab_kc, static_cast<const int *>(gen_flag), launch_id, 1, int(CLS_GEN));
        HIP_TRY(hipGetLastError());
    }
    {
        const int64_t lds_k1 = slice_bytes_for(ls.mmax, ls.r1, ls.tab, 0);
        int per_cu = 0;
        HIP_TRY(ctx->occupancy(reinterpret_cast<const void *>(halda_solve_kernel), lds_k1, &per_cu));
        const int64_t cap = wide ? int64_t(ctx->cus) * per_cu : int64_t(ctx->cus);
        const int grid = int(std::max<int64_t>(1, std::min<int64_t>(cap, in.n_inst)));
        hipLaunchKernelGGL(halda_solve_kernel, dim3(grid), dim3(64), size_t(lds_k1), stream, in, out, cls, ls.mmax,
                           ls.r1, ls.tab, 0, static_cast<const int *>(hb_flag), launch_id, int(!wide),
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

// The fused sweep's launch sequence for one batch shape, derived from the shapes alone (no HIP call):
// which kernels, their grids and LDS slices, and the kernel arguments but for the per-launch scratch
// fields (fflag, hb_flag, launch_id, want), which run_sweep fills. sweep_fleets plans and runs in one
// go; a prepared plan (halda_fleets_plan_create) is planned once and run per launch.
enum SweepKind { kRegAlone, kRegGated, kRegBig, kTablesAlone, kSegGated, kKslotGated };

struct SweepPlan {
    SweepArgs A;
    SlotArgs SA;
    SweepKind kind;
    bool scratch;      // per-fleet flags / hand-back flag of the stream's slot in use
    int nf;
    int64_t lds;       // the first launch's dynamic LDS (k-slot / segment / table kernel)
    int64_t slice;     // the table kernel's LDS slice
    unsigned grid1;    // the first launch's grid
    unsigned block1;   // its workgroup size
    unsigned grid2;    // the gated second launch's grid (0: none)
    const void *fn1;   // first kernel (for the occupancy / LDS attribute)
};

int plan_sweep(Ctx *c, const halda_model &model, const halda_fleets &F, const int32_t *kh, int n_k,
               const halda_fleet_result &out, SweepPlan *P) {
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
        // a fleet of M >= min_devices devices has R + 1 <= r1 rows of odd stride <= odd_stride(r1)
        SA.tab[q] = kh[j] > 1 && W > F.min_devices ? mmax * odd_stride(SA.r1[q]) : 0;
        SA.off[q] = int(kslot_lds);
        kslot_lds += (64 / kSegLanes) * kslot_slice_bytes(mmax, SA.tab[q]);
    }
    bool kslot_all = true;  // every k that is open for some fleet has a slot
    for (int j = 0, q = 0; j < n_k; ++j) {
        const int W = model.L / kh[j];
        if (!(W < 1000000) || W < F.min_devices) continue;
        kslot_all = kslot_all && q < SA.n_slot && SA.j[q] == j;
        ++q;
    }
    // region 0 holds, one after another, the device records (read before any table is written), the
    // tables, and the pick area (written after the last table read): as large as the largest of them
    const int64_t pick_bytes = int64_t(64 / kSegLanes) * SA.n_slot * int64_t(sizeof(SlotPick));
    kslot_lds = std::max<int64_t>({kslot_lds, pick_bytes, int64_t(sizeof(KslotRecs))});
    SA.pick_off = 0;
    SA.rec_off = 0;
    // the threshold scan of the slot with the largest tables (C2: k = 2, the workgroup's critical path)
    // is split over kslot_split waves: the slot's own and, first thing after the tables, the waves of
    // the lightest other slots (no tables: k = 1 / W = M; else the smallest tables) -- an extra wave
    // only when there is no other slot
    SA.helper = -1;
    SA.n_parts = 0;
    if (c->kslot_split >= 2) {
        int r1 = 0;
        for (int q = 0; q < SA.n_slot; ++q)
            if (SA.tab[q] > 0 && SA.r1[q] > r1) {
                r1 = SA.r1[q];
                SA.helper = q;
            }
    }
    if (SA.helper >= 0) {
        // helpers: the lightest other slots (no tables, then the smallest; ties: the later slot)
        int used = 0;
        for (int h = 0; h < c->kslot_split - 1; ++h) {
            int pick = -1, light = 1 << 30;
            for (int q = 0; q < SA.n_slot; ++q) {
                const int work = SA.tab[q] > 0 ? SA.r1[q] : 0;
                bool taken = q == SA.helper;
                for (int u = 0; u < used; ++u) taken = taken || SA.part_wave[u] == q;
                if (!taken && work <= light) {
                    light = work;
                    pick = q;
                }
            }
            if (pick < 0) break;
            SA.part_wave[used++] = pick;
        }
        if (used == 0) {  // no other slot: one extra wave takes part 2
            if (SA.n_slot < kMaxSlots) SA.part_wave[used++] = SA.n_slot;
            else SA.helper = -1;
        }
        SA.n_parts = used + 1;
    }
    // the leaf checks of an optimistic part 1 (kslot_check): the table slot with the smallest tables
    // other than the split one (it ends its own solve first), else the other no-table slot, else the
    // helper itself
    SA.check_wave = -1;
    if (SA.helper >= 0) {
        SA.check_wave = SA.part_wave[0];
        int best = 1 << 30;
        for (int q = 0; q < SA.n_slot; ++q) {
            if (q == SA.helper || q == SA.part_wave[0]) continue;
            const int work = SA.tab[q] > 0 ? SA.r1[q] : (1 << 20);  // a no-table slot: its k = 1 greedy
            if (work < best) {
                best = work;
                SA.check_wave = q;
            }
        }
    }
    SA.crit_w4 = c->kslot_crit_w4;
    SA.cut8 = c->kslot_cut8;
    SA.opt = c->kslot_opt ? 1 : 0;
    kslot_lds = align16(kslot_lds);
    SA.split_off = int(kslot_lds);
    if (SA.helper >= 0) kslot_lds += int64_t(64 / kSegLanes) * int64_t(sizeof(SplitArea));
    kslot_lds = align16(kslot_lds);
    kslot_lds += c->kslot_pad;
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
    SweepPlan &p = *P;
    p = SweepPlan{};
    p.nf = nf;
    p.slice = slice;
    p.scratch = !(reg_mode && !gate);
    SweepArgs &A = p.A;
    static_cast<halda_model &>(A.Mo) = model;
    A.Mo.bvo = model_bvo(model);
    A.F = F;
    for (int j = 0; j < n_k; ++j) {
        A.ks[j] = kh[j];
        A.Ws[j] = kh[j] != 0 ? model.L / kh[j] : 0;
    }
    A.n_k = n_k;
    A.out = FleetOut(out);
    A.outs = (out.obj_by_k ? kOutObk : 0) | (out.status ? kOutSt : 0) | (out.x ? kOutX : 0) | (out.c ? kOutC : 0) |
             (c->x_zero ? kOutXZ : 0);
    A.x_off = out.x_off;
    A.xstride = 7 * int64_t(std::max(mmax, 1)) + 1;
    A.mmax = mmax;
    A.uM = F.min_devices == F.max_devices ? F.max_devices : 0;
    A.k1dp = c->k1_force_dp ? 1 : 0;
    A.r1max = int(r1max);
    A.tab = int(tab);
    A.tab_kc = int(tab_kc);
    p.SA = SA;
    const unsigned cap_cus = unsigned(std::min<int64_t>(c->cus, nf));
    if (kslot) {
        p.kind = kKslotGated;
        p.fn1 = reinterpret_cast<const void *>(halda_sweep_kslot_kernel);
        p.lds = kslot_lds;
        p.grid1 = unsigned((int64_t(nf) + 64 / kSegLanes - 1) / (64 / kSegLanes));
        p.block1 = unsigned(64 * kslot_waves(SA));
        p.grid2 = cap_cus;
    } else if (seg) {
        p.kind = kSegGated;
        p.fn1 = reinterpret_cast<const void *>(halda_sweep_seg_kernel);
        p.lds = seg_lds;
        int per_cu = 0;
        HIP_TRY(c->occupancy(p.fn1, seg_lds, &per_cu));
        const int64_t nw = (int64_t(nf) + 64 / kSegLanes - 1) / (64 / kSegLanes);
        p.grid1 = unsigned(std::max<int64_t>(1, std::min<int64_t>(int64_t(c->cus) * per_cu, nw)));
        p.block1 = 64;
        p.grid2 = cap_cus;
    } else if (fits && (tables_first || small_tables)) {
        // small batches (a single halda_solve): one launch with the table slice instead of two
        p.kind = kTablesAlone;
        p.fn1 = reinterpret_cast<const void *>(halda_sweep_tables_kernel);
        p.lds = slice;
        int per_cu = 0;
        HIP_TRY(c->occupancy(p.fn1, slice, &per_cu));
        p.grid1 = unsigned(std::max<int64_t>(1, std::min<int64_t>(int64_t(c->cus) * per_cu, nf)));
        p.block1 = 64;
    } else {
        p.fn1 = reinterpret_cast<const void *>(halda_sweep_kernel);
        p.grid1 = unsigned((nf + kSweepWavesPerBlock - 1) / kSweepWavesPerBlock);
        p.block1 = 64 * kSweepWavesPerBlock;
        if (!gate) {
            p.kind = kRegAlone;
        } else if (fits) {  // flagged fleets are rare (fast-path fallbacks): one wave per CU is plenty
            p.kind = kRegGated;
            int per_cu = 0;
            HIP_TRY(c->occupancy(reinterpret_cast<const void *>(halda_sweep_tables_kernel), slice, &per_cu));
            p.grid2 = unsigned(std::max<int64_t>(1, std::min<int64_t>(tables_first ? int64_t(c->cus) * per_cu
                                                                                   : int64_t(c->cus), nf)));
        } else {
            p.kind = kRegBig;
            A.gstride = (slice + 255) & ~int64_t(255);
            int per_cu = 0;
            HIP_TRY(c->occupancy(reinterpret_cast<const void *>(halda_sweep_big_kernel), 0, &per_cu));
            p.grid2 = unsigned(std::max<int64_t>(
                1, std::min<int64_t>({int64_t(c->cus) * per_cu, int64_t(nf), kGlobalTableBudget / A.gstride})));
        }
    }
    if (p.kind == kKslotGated) {
        int per_cu = 0;
        HIP_TRY(c->occupancy(p.fn1, p.lds, &per_cu));
        if (std::getenv("HALDA_DEBUG_PLAN")) {  // diagnostic: the k-slot launch's LDS and residency
            int steps_cu = 0;
            (void)c->ensure_lds(reinterpret_cast<const void *>(halda_sweep_kslot_steps_kernel), p.lds);
            (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &steps_cu, reinterpret_cast<const void *>(halda_sweep_kslot_steps_kernel), int(p.block1),
                size_t(p.lds));
            std::fprintf(stderr, "halda plan: k-slot lds %lld B, block %u, per CU %d (steps kernel %d)\n",
                         (long long)p.lds, p.block1, per_cu, steps_cu);
        }
    }
    if (p.kind == kKslotGated || p.kind == kSegGated)
        HIP_TRY(c->occupancy(reinterpret_cast<const void *>(halda_sweep_tables_kernel), slice, nullptr));
    return HALDA_OK;
}

// Enqueue a planned sweep on stream s: the stream's scratch slot (when the plan uses scratch), the
// first launch and the gated table launch behind it (global tables: after the previous launch on them).
int run_sweep(Ctx *c, SweepPlan &p, hipStream_t s) {
    SweepArgs &A = p.A;
    Ctx::SweepSlot *slot = nullptr;
    if (p.scratch) {
        const int rc = sweep_slot(c, s, p.nf, &slot);
        if (rc != HALDA_OK) return rc;
    }
    A.fflag = p.scratch ? slot->fflag : nullptr;
    A.hb_flag = p.scratch ? slot->hb : c->hb_flag;
    A.launch_id = ++c->launch_id;
    A.want = 0;
    c->fleet_timed = false;
    c->have_lowered = false;
    if (p.lds > 0) HIP_TRY(Ctx::ensure_lds(p.fn1, p.lds));
    if (c->timing) HIP_TRY(hipEventRecord(c->evf0, s));
    switch (p.kind) {
        case kKslotGated:
            hipLaunchKernelGGL(halda_sweep_kslot_kernel, dim3(p.grid1), dim3(p.block1), size_t(p.lds), s, A, p.SA);
            break;
        case kSegGated:
            hipLaunchKernelGGL(halda_sweep_seg_kernel, dim3(p.grid1), dim3(p.block1), size_t(p.lds), s, A);
            break;
        case kTablesAlone:
            hipLaunchKernelGGL(halda_sweep_tables_kernel, dim3(p.grid1), dim3(p.block1), size_t(p.lds), s, A);
            break;
        default:
            hipLaunchKernelGGL(halda_sweep_kernel, dim3(p.grid1), dim3(p.block1), 0, s, A);
            break;
    }
    HIP_TRY(hipGetLastError());
    const bool two = p.kind == kKslotGated || p.kind == kSegGated || p.kind == kRegGated || p.kind == kRegBig;
    if (two) {
        if (c->timing) HIP_TRY(hipEventRecord(c->evfm, s));
        A.want = 1;  // the fleets flagged above, gated on the hand-back flag
        if (p.kind == kRegBig) {
            const size_t gneed = size_t(A.gstride) * size_t(p.grid2);
            if (gneed > c->gtab_bytes) {
                if (c->gtab) HIP_TRY(hipFree(c->gtab));
                c->gtab = nullptr;
                c->gtab_bytes = 0;
                HIP_TRY(hipMalloc(&c->gtab, gneed));
                c->gtab_bytes = gneed;
            }
            // the global tables are per context (not per stream slot: up to 2 GiB each), so this launch
            // runs after the previous user of them on another stream (a sweep's or launch()'s big launch)
            const int rc = order_after_previous(c, s);
            if (rc != HALDA_OK) return rc;
            A.gtab = static_cast<unsigned char *>(c->gtab);
            hipLaunchKernelGGL(halda_sweep_big_kernel, dim3(p.grid2), dim3(64), 0, s, A);
        } else {
            HIP_TRY(Ctx::ensure_lds(reinterpret_cast<const void *>(halda_sweep_tables_kernel), p.slice));
            hipLaunchKernelGGL(halda_sweep_tables_kernel, dim3(p.grid2), dim3(64), size_t(p.slice), s, A);
        }
        HIP_TRY(hipGetLastError());
    }
    if (c->timing) {
        HIP_TRY(hipEventRecord(c->evf1, s));
        c->fleet_timed = true;
    }
    c->fleet_two = two;
    c->fleet_reg_alone = p.kind == kRegAlone;
    c->fleet_seg = p.kind == kSegGated;
    c->fleet_kslot = p.kind == kKslotGated;
    c->last_fleet_fused = true;
    return HALDA_OK;
}

// The last call's arguments and plan: a caller repeating a call on the same buffers (a single
// halda_solve's staging, a re-profiled stream) is not re-planned.
struct SweepKey {
    halda_model model;
    halda_fleets F;
    halda_fleet_result out;
    int32_t ks[64];
    int n_k, path_gen;
    bool x_zero;
};

int cached_plan(Ctx *c, const halda_model &model, const halda_fleets &F, const int32_t *kh, int n_k,
                const halda_fleet_result &out, SweepPlan **plan) {
    static thread_local SweepKey last_key;
    static thread_local SweepPlan last_plan;
    static thread_local uint64_t last_ctx = 0;  // Ctx::uid
    SweepKey k;
    std::memset(&k, 0, sizeof k);
    k.model = model;
    k.F = F;
    k.out = out;
    std::memcpy(k.ks, kh, sizeof(int32_t) * size_t(n_k));
    k.n_k = n_k;
    k.path_gen = c->path_gen;
    k.x_zero = c->x_zero;
    if (last_ctx != c->uid || std::memcmp(&k, &last_key, sizeof k) != 0) {
        last_ctx = 0;
        const int rc = plan_sweep(c, model, F, kh, n_k, out, &last_plan);
        if (rc != HALDA_OK) return rc;
        last_key = k;
        last_ctx = c->uid;
    }
    *plan = &last_plan;
    return HALDA_OK;
}

int sweep_fleets(Ctx *c, const halda_model &model, const halda_fleets &F, const int32_t *kh, int n_k,
                 const halda_fleet_result &out, hipStream_t s) {
    SweepPlan *p = nullptr;
    const int rc = cached_plan(c, model, F, kh, n_k, out, &p);
    if (rc != HALDA_OK) return rc;
    return run_sweep(c, *p, s);
}

// One fleet through the resident wave (halda_resident_kernel), synchronously: the plan's arguments into
// the mailbox, the wave (re)launched when no launch of it is running, seq bumped, ack awaited. The
// fleet's table and results are the caller's fine-grained pinned buffers (device addresses in A).
// *done = false when the plan is not a register-only sweep of one fleet, or when the wave gave no answer
// in time and was stopped (the caller launches the sweep itself; the resident path is off from then on).
// *retry = true when the wave could not even be stopped: its pinned buffer is retired (kept allocated,
// never reused) and the caller redoes the whole call on a fresh one.
constexpr uint32_t kResidentIdleTicks = 200000;  // 2 ms of the 100 MHz clock without a request

// Stop the resident wave and wait (at most `budget`) until it has left: true when it has (or none ran).
bool resident_stop(Ctx *c, std::chrono::milliseconds budget) {
    if (!c->rbox || !c->rlive) return true;
    __atomic_store_n(&c->rbox->stop, 1u, __ATOMIC_SEQ_CST);
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t q;
    while ((q = hipEventQuery(c->rdone)) == hipErrorNotReady) {
        if (std::chrono::steady_clock::now() - t0 > budget) return false;
        std::this_thread::yield();
    }
    c->rlive = false;
    __atomic_store_n(&c->rbox->stop, 0u, __ATOMIC_SEQ_CST);  // the next launch stays until told
    return true;
}

int resident_sweep(Ctx *c, const SweepPlan &p, bool *done, bool *retry) {
    *done = false;
    *retry = false;
    if (!c->resident || p.kind != kRegAlone || p.nf != 1 || p.A.uM <= 0 || p.A.uM > kK1MaxM || p.A.k1dp) return HALDA_OK;
    if (!c->rbox) {
        HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&c->rbox), sizeof(ResidentBox),
                              hipHostMallocMapped | hipHostMallocCoherent));
        std::memset(static_cast<void *>(c->rbox), 0, sizeof(ResidentBox));
        HIP_TRY(hipHostGetDevicePointer(&c->rbox_dev, c->rbox, 0));
        HIP_TRY(hipStreamCreateWithFlags(&c->rstream, hipStreamNonBlocking));
        HIP_TRY(hipEventCreateWithFlags(&c->rdone, hipEventDisableTiming));
        c->rseq = 0;
    }
    ResidentBox *box = c->rbox;
    SweepArgs A = p.A;
    A.fflag = nullptr;
    A.hb_flag = c->hb_flag;
    A.launch_id = ++c->launch_id;
    A.want = 0;
    std::memcpy(static_cast<void *>(&box->req), &A, sizeof A);
    auto launch = [&](uint32_t last) -> int {
        ResidentArgs R;
        R.box = static_cast<ResidentBox *>(c->rbox_dev);
        R.last = last;
        R.idle_ticks = kResidentIdleTicks;
        hipLaunchKernelGGL(halda_resident_kernel, dim3(1), dim3(64), 0, c->rstream, R);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(c->rdone, c->rstream));
        c->rlive = true;
        return HALDA_OK;
    };
    if (!c->rlive || hipEventQuery(c->rdone) == hipSuccess) {
        const int rc = launch(c->rseq);
        if (rc != HALDA_OK) return rc;
    }
    const uint32_t want = ++c->rseq;
    // after the request (x86: stores in order); the fault-injection mode never posts it
    if (!c->resident_drop) __atomic_store_n(&box->seq, want, __ATOMIC_SEQ_CST);
    // the answer; a wave that left (idle timeout) between its last poll and this request is relaunched
    const auto t0 = std::chrono::steady_clock::now();
    const auto limit = c->resident_drop ? std::chrono::milliseconds(20) : std::chrono::milliseconds(5000);
    for (uint64_t spin = 1;; ++spin) {
        if (__atomic_load_n(&box->ack, __ATOMIC_ACQUIRE) == want) break;
        if ((spin & 255) == 0) {
            if (hipEventQuery(c->rdone) == hipSuccess && __atomic_load_n(&box->ack, __ATOMIC_ACQUIRE) != want) {
                const int rc = launch(want - 1);
                if (rc != HALDA_OK) return rc;
            }
            if (std::chrono::steady_clock::now() - t0 > limit) {
                // no answer: never again on this context. The wave (or a late launch of it) still sees
                // request `want` pending and would write its results into the pinned buffer later, so it
                // is stopped and awaited before that buffer is touched again; then this call launches.
                c->resident = false;
                if (resident_stop(c, std::chrono::milliseconds(5000))) return HALDA_OK;
                c->retired.push_back(c->pinned);  // still the wave's: keep it allocated, never reuse it
                c->pinned = nullptr;
                c->pinned_dev = nullptr;
                c->pinned_bytes = 0;
                *retry = true;
                return HALDA_OK;
            }
        }
    }
    *done = true;
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

// The steps of latency mode, shared by the RCCL entry (one rank: this process's) and the one-device
// emulation of `world` ranks (tests, bench): per rank the sub-sweep of its k's and halda_shard_kernel
// mode 0, all-reduce MIN obj_value, mode 1, all-reduce MIN best_k, mode 2, then (one RCCL group) SUM w,
// SUM n, MIN obj_by_k, MAX status, and the final kernel. `ar(field, count)` performs one all-reduce (or
// opens / closes the group) over the ranks' `o` arrays.
enum ShardField { kShObj, kShBestK, kShGroupStart, kShW, kShN, kShObk, kShSt, kShGroupEnd };

struct ShardRank {
    int rank = 0;
    halda_fleet_result o = {};    // this rank's copy of the full result
    halda_fleet_result sub = {};  // its sub-sweep's results (its k's only)
    std::vector<int32_t> mine;    // ks[rank], ks[rank + world], ...
};

constexpr int kEmuMaxWorld = 16;
struct EmuReduce {
    int world;
    int field;
    int64_t count;
    void *p[kEmuMaxWorld];
};

// One emulated all-reduce: element i of every virtual rank's buffer becomes the MIN / SUM / MAX over
// the ranks (the RCCL operation of that field), in place.
__global__ __launch_bounds__(256) void halda_emu_allreduce_kernel(EmuReduce E) {
    const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (i >= E.count) return;
    if (E.field == kShObj || E.field == kShObk) {
        double m = static_cast<const double *>(E.p[0])[i];
        for (int r = 1; r < E.world; ++r) {
            const double v = static_cast<const double *>(E.p[r])[i];
            m = v < m ? v : m;
        }
        for (int r = 0; r < E.world; ++r) static_cast<double *>(E.p[r])[i] = m;
    } else {
        int32_t m = static_cast<const int32_t *>(E.p[0])[i];
        for (int r = 1; r < E.world; ++r) {
            const int32_t v = static_cast<const int32_t *>(E.p[r])[i];
            m = E.field == kShBestK ? (v < m ? v : m) : E.field == kShSt ? (v > m ? v : m) : m + v;
        }
        for (int r = 0; r < E.world; ++r) static_cast<int32_t *>(E.p[r])[i] = m;
    }
}

// Devices in the batch: n_fleets * M for one fleet size, else dev_off[n_fleets] read back (synchronous).
int shard_device_count(const halda_fleets &F, hipStream_t s, int64_t *nd) {
    const int64_t nf = F.n_fleets;
    *nd = nf * F.max_devices;
    if (F.min_devices != F.max_devices) {
        HIP_TRY(hipMemcpyAsync(nd, F.dev_off + nf, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    return HALDA_OK;
}

template <class AR>
int shard_steps(Ctx *c, const halda_model &model, const halda_fleets &F, const int32_t *ks, int n_k, int world,
                std::vector<ShardRank> &R, hipStream_t s, AR &&ar) {
    const halda_fleet_result &out = R[0].o;
    if (out.x || out.c) return fail(HALDA_E_ARG, "halda_solve_fleets_sharded: x / c are not gathered (pass NULL)");
    if (!out.best_k || !out.obj_value || !out.w || !out.n) return fail(HALDA_E_ARG, "halda_fleet_result: NULL");
    const int64_t nf = F.n_fleets;
    if (nf <= 0) return HALDA_OK;
    if (n_k <= 0 || n_k > 1024) return fail(HALDA_E_ARG, "n_k must be in 1..1024");
    for (int j = 0; j < n_k; ++j)
        if (ks[j] < 1 || (j && ks[j] <= ks[j - 1])) return fail(HALDA_E_ARG, "ks must be ascending, unique, > 0");
    int64_t nd = 0;
    {
        const int rc = shard_device_count(F, s, &nd);
        if (rc != HALDA_OK) return rc;
    }
    // rank-local sub-sweep results in the context's shard scratch (one block per rank state)
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off += (bytes + 255) & ~size_t(255); return o; };
    std::vector<size_t> o_bk, o_obj, o_w, o_n, o_obk, o_st;
    for (auto &r : R) {
        r.mine.clear();
        for (int j = r.rank; j < n_k; j += world) r.mine.push_back(ks[j]);  // as halda_solve_distributed deals them
        const size_t nsub = std::max<size_t>(r.mine.size(), 1);
        o_bk.push_back(take(4 * nf));
        o_obj.push_back(take(8 * nf));
        o_w.push_back(take(4 * size_t(nd)));
        o_n.push_back(take(4 * size_t(nd)));
        o_obk.push_back(take(8 * nf * nsub));
        o_st.push_back(take(4 * nf * nsub));
    }
    if (off > c->shard_bytes) {
        if (c->shard) HIP_TRY(hipFree(c->shard));
        c->shard = nullptr;
        c->shard_bytes = 0;
        HIP_TRY(hipMalloc(&c->shard, off));
        c->shard_bytes = off;
    }
    char *base = static_cast<char *>(c->shard);
    for (size_t i = 0; i < R.size(); ++i) {
        halda_fleet_result &sub = R[i].sub;
        sub = {};
        sub.best_k = reinterpret_cast<int32_t *>(base + o_bk[i]);
        sub.obj_value = reinterpret_cast<double *>(base + o_obj[i]);
        sub.w = reinterpret_cast<int32_t *>(base + o_w[i]);
        sub.n = reinterpret_cast<int32_t *>(base + o_n[i]);
        sub.obj_by_k = out.obj_by_k ? reinterpret_cast<double *>(base + o_obk[i]) : nullptr;
        sub.status = out.status ? reinterpret_cast<int32_t *>(base + o_st[i]) : nullptr;
    }
    {
        const int rc = order_after_previous(c, s);  // the shard scratch is per context
        if (rc != HALDA_OK) return rc;
    }
    for (auto &r : R)
        if (!r.mine.empty()) {
            const int rc = halda_solve_fleets(c, &model, &F, r.mine.data(), int32_t(r.mine.size()), &r.sub, s);
            if (rc != HALDA_OK) return rc;
        }
    auto modes = [&](int mode) -> int {
        for (auto &r : R) {
            hipLaunchKernelGGL(halda_shard_kernel, dim3(unsigned(nf)), dim3(64), 0, s, mode, int(n_k),
                               int(r.mine.size()), r.rank, world, F.dev_off, r.sub, r.o);
            HIP_TRY(hipGetLastError());
        }
        return HALDA_OK;
    };
    int rc = modes(0);
    if (rc == HALDA_OK) rc = ar(kShObj, size_t(nf));
    if (rc == HALDA_OK) rc = modes(1);
    if (rc == HALDA_OK) rc = ar(kShBestK, size_t(nf));
    if (rc == HALDA_OK) rc = modes(2);
    if (rc == HALDA_OK) rc = ar(kShGroupStart, 0);
    if (rc == HALDA_OK) rc = ar(kShW, size_t(nd));
    if (rc == HALDA_OK) rc = ar(kShN, size_t(nd));
    if (rc == HALDA_OK && out.obj_by_k) rc = ar(kShObk, size_t(nf) * n_k);
    if (rc == HALDA_OK && out.status) rc = ar(kShSt, size_t(nf) * n_k);
    if (rc == HALDA_OK) rc = ar(kShGroupEnd, 0);
    if (rc != HALDA_OK) return rc;
    for (auto &r : R) {
        hipLaunchKernelGGL(halda_shard_final_kernel, dim3(unsigned((nf + 255) / 256)), dim3(256), 0, s, int(nf), r.o);
        HIP_TRY(hipGetLastError());
    }
    return HALDA_OK;
}

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
    const char *fp = std::getenv("HALDA_FLEETS_PATH");
    c->fleets_fused = !(fp && std::strcmp(fp, "csr") == 0);
    c->seg_sweep = !(fp && std::strcmp(fp, "wave") == 0);
    const char *hp = std::getenv("HALDA_HOST_PATH");  // diagnostic A/B of the small synchronous call
    c->host_copy = hp && std::strcmp(hp, "copy") == 0;
    const char *rs = std::getenv("HALDA_RESIDENT");
    c->resident = !(rs && std::strcmp(rs, "0") == 0);
    const char *fs = std::getenv("HALDA_FUSED_SCREEN");  // A/B: the screen launch before a settled batch's k = 1 kernel
    c->fused_screen = !(fs && std::strcmp(fs, "0") == 0);
    const char *kw = std::getenv("HALDA_KSLOT_CRIT_W4");  // diagnostic A/B of the critical slot's table share
    if (kw && std::atoi(kw) > 0) c->kslot_crit_w4 = std::atoi(kw);
    const char *kc8 = std::getenv("HALDA_KSLOT_CUT8");  // diagnostic A/B of the split scan's cut
    if (kc8 && std::atoi(kc8) >= 1 && std::atoi(kc8) <= 7) c->kslot_cut8 = std::atoi(kc8);
    const char *kp = std::getenv("HALDA_KSLOT_LDS_PAD");
    c->kslot_pad = kp ? std::max(0, std::atoi(kp)) : 0;
    const char *rt = std::getenv("HALDA_RESIDENT_TEST");
    c->resident_drop = rt && std::strcmp(rt, "drop") == 0;
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

int halda_resident_release(void *ctx) {
    Ctx *c = static_cast<Ctx *>(ctx);
    if (!c) return fail(HALDA_E_ARG, "null context");
    if (!resident_stop(c, std::chrono::milliseconds(5000)))
        return fail(HALDA_E_HIP, "resident solver: the wave did not leave within 5 s");
    return HALDA_OK;
}

int halda_host_alloc(size_t bytes, void **ptr) {
    if (!ptr || bytes == 0) return fail(HALDA_E_ARG, "halda_host_alloc: NULL ptr or zero bytes");
    *ptr = nullptr;
    HIP_TRY(hipHostMalloc(ptr, bytes, hipHostMallocDefault));
    std::lock_guard<std::mutex> lock(g_host_mu);
    g_host_blocks.emplace_back(reinterpret_cast<uintptr_t>(*ptr), bytes);
    return HALDA_OK;
}

void halda_host_free(void *ptr) {
    if (!ptr) return;
    {
        std::lock_guard<std::mutex> lock(g_host_mu);
        for (size_t i = 0; i < g_host_blocks.size(); ++i)
            if (g_host_blocks[i].first == reinterpret_cast<uintptr_t>(ptr)) {
                g_host_blocks.erase(g_host_blocks.begin() + i);
                break;
            }
    }
    (void)hipHostFree(ptr);
}

void halda_free(void *ctx) {
    Ctx *c = static_cast<Ctx *>(ctx);
    if (!c) return;
    for (CtxHandle *h : c->handles) h->c = nullptr;  // plans / groups outliving the context fail cleanly
    c->handles.clear();
    if (c->rbox) {
        if (c->rlive) {  // the resident wave leaves at its next poll
            __atomic_store_n(&c->rbox->stop, 1u, __ATOMIC_SEQ_CST);
            (void)hipEventSynchronize(c->rdone);
        }
        (void)hipHostFree(c->rbox);
    }
    for (void *b : c->retired) (void)hipHostFree(b);  // the wave that held them has left (above)
    if (c->rdone) (void)hipEventDestroy(c->rdone);
    if (c->rstream) (void)hipStreamDestroy(c->rstream);
    (void)hipSetDevice(c->device);
    if (c->scratch) (void)hipFree(c->scratch);
    if (c->pinned) (void)hipHostFree(c->pinned);
    if (c->work) (void)hipFree(c->work);
    if (c->hb_flag) (void)hipFree(c->hb_flag);
    if (c->fleet_scratch) (void)hipFree(c->fleet_scratch);
    if (c->gtab) (void)hipFree(c->gtab);
    for (auto &x : c->sws) {
        if (x.fflag) (void)hipFree(x.fflag);
        if (x.cls) (void)hipFree(x.cls);
        if (x.hb) (void)hipFree(x.hb);
        if (x.ev) (void)hipEventDestroy(x.ev);
    }
    if (c->shard) (void)hipFree(c->shard);
    if (c->emu) (void)hipFree(c->emu);
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

int halda_solve_batch_device_settled(void *ctx, const halda_batch *in, halda_result *out, const uint8_t *settled,
                                     void *stream) {
    Ctx *c = static_cast<Ctx *>(ctx);
    if (!c || !in || !out) return fail(HALDA_E_ARG, "NULL ctx/in/out");
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->stream;
    return launch(c, *in, *out, s, settled);
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
    if (c->fused_last) {  // no screen launch: the settled k = 1 kernel from the start
        HIP_TRY(hipEventElapsedTime(&b, c->ev0, c->evs));
    } else {
        HIP_TRY(hipEventElapsedTime(&a, c->ev0, c->evk));
        HIP_TRY(hipEventElapsedTime(&b, c->evk, c->evs));
    }
    HIP_TRY(hipEventElapsedTime(&d, c->evs, c->ev1));
    ms3[0] = a;
    ms3[1] = b;
    ms3[2] = d;
    return HALDA_OK;
}

int halda_set_fleets_path(void *ctx, int path) {
    Ctx *c = static_cast<Ctx *>(ctx);
    if (!c) return fail(HALDA_E_ARG, "NULL ctx");
    if (path < 0 || path > 6)
        return fail(HALDA_E_ARG, "path must be 0 (CSR), 1 (fused), 2 (fused, one fleet per wave), 3 (fused, k = 1 "
                                 "by DP), 4 (fused, segment kernel instead of the k-slot kernel), 5 (fused, the "
                                 "k-slot scan unsplit), 6 (fused, the k-slot split scan in sequential order)");
    c->fleets_fused = path != 0;
    c->seg_sweep = path == 1 || path == 4 || path == 5 || path == 6;
    c->kslot_sweep = path == 1 || path == 5 || path == 6;
    c->k1_force_dp = path == 3;
    c->kslot_split = path == 5 ? 0 : 2;
    c->kslot_opt = path != 6;
    ++c->path_gen;
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
int halda_debug_scanprof(unsigned long long *out, int n_wave) {
    const int n = std::min(n_wave, kStampInst);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_halda_scanprof), sizeof(unsigned long long) * kScanProf * n));
    return n;
}
int halda_debug_dump(double *out) {
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_halda_dump), sizeof(double) * kDumpFleets * kDumpDev * kDumpE * 2));
    return kDumpFleets;
}
#endif

}  // extern "C"

namespace {
// Argument checks shared by halda_solve_fleets and halda_fleets_plan_create (HALDA_OK: go on).
int check_fleets_args(const halda_model *model, const halda_fleets *fleets, const int32_t *ks, int32_t n_k,
                      const halda_fleet_result *out) {
    const halda_fleets &F = *fleets;
    if (n_k <= 0 || n_k > 1024) return fail(HALDA_E_ARG, "n_k must be in 1..1024");
    if (F.min_devices < 1 || F.max_devices < F.min_devices || F.max_devices > 4096)
        return fail(HALDA_E_ARG, "halda_fleets: need 1 <= min_devices <= max_devices <= 4096");
    if (!F.dev_off || !F.os_class || !F.flags || !F.scpu_b1 || !F.sgpu_b1 || !F.T_cpu || !F.T_gpu ||
        !F.t_kvcpy_cpu || !F.t_kvcpy_gpu || !F.t_ram2vram || !F.t_vram2ram || !F.t_comm || !F.s_disk ||
        !F.d_avail_ram || !F.c_cpu || !F.c_gpu || !F.d_avail_cuda || !F.d_avail_metal || !F.swap)
        return fail(HALDA_E_ARG, "halda_fleets has a NULL array");
    if (!out->best_k || !out->obj_value || !out->w || !out->n) return fail(HALDA_E_ARG, "halda_fleet_result: NULL");
    if (model->L < 1) return fail(HALDA_E_ARG, "model.L < 1");
    // ks (host memory): ascending, unique, positive
    for (int j = 0; j < n_k; ++j)
        if (ks[j] < 1 || (j && ks[j] <= ks[j - 1])) return fail(HALDA_E_ARG, "ks must be ascending, unique, > 0");
    return HALDA_OK;
}

// A prepared k-sweep (halda_fleets_plan_create): the fused sweep's plan, or, when the context runs
// halda_solve_fleets another way (the CSR pipeline, more than 64 k), the call's arguments.
struct FleetsPlan : CtxHandle {
    int gen = 0;  // the context's path_gen when planned
    bool fused = false;
    SweepPlan p;
    halda_model model;
    halda_fleets F;
    std::vector<int32_t> ks;
    halda_fleet_result out;
};

// (Re)derive a plan's launch sequence for its context's current path.
int replan(FleetsPlan *P) {
    Ctx *c = P->c;
    P->gen = c->path_gen;
    P->fused = P->F.n_fleets > 0 && c->fleets_fused && P->ks.size() <= 64;
    if (!P->fused) return HALDA_OK;
    return plan_sweep(c, P->model, P->F, P->ks.data(), int(P->ks.size()), P->out, &P->p);
}
}  // namespace

extern "C" {

int halda_solve_fleets(void *ctx, const halda_model *model, const halda_fleets *fleets, const int32_t *ks,
                       int32_t n_k, halda_fleet_result *out, void *stream) {
    Ctx *c = static_cast<Ctx *>(ctx);
    if (!c || !model || !fleets || !ks || !out) return fail(HALDA_E_ARG, "NULL ctx/model/fleets/ks/out");
    const halda_fleets &F = *fleets;
    if (F.n_fleets <= 0) return HALDA_OK;
    {
        const int rc = check_fleets_args(model, fleets, ks, n_k, out);
        if (rc != HALDA_OK) return rc;
    }
    int cur_dev = -1;
    if (hipGetDevice(&cur_dev) != hipSuccess || cur_dev != c->device) HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->stream;
    const int32_t *kh = ks;
    // the fused sweep orders itself: per-stream scratch slots, and order_after_previous before a launch
    // on the context's global tables
    if (c->fleets_fused && n_k <= 64) return sweep_fleets(c, *model, F, ks, n_k, *out, s);
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

int halda_fleets_plan_create(void *ctx, const halda_model *model, const halda_fleets *fleets, const int32_t *ks,
                             int32_t n_k, const halda_fleet_result *out, void **plan) {
    Ctx *c = static_cast<Ctx *>(ctx);
    if (!c || !model || !fleets || !ks || !out || !plan) return fail(HALDA_E_ARG, "NULL ctx/model/fleets/ks/out/plan");
    if (fleets->n_fleets > 0) {
        const int rc = check_fleets_args(model, fleets, ks, n_k, out);
        if (rc != HALDA_OK) return rc;
    }
    HIP_TRY(hipSetDevice(c->device));
    FleetsPlan *P = new FleetsPlan();
    P->c = c;
    P->model = *model;
    P->F = *fleets;
    P->ks.assign(ks, ks + std::max(n_k, 0));
    P->out = *out;
    const int rc = replan(P);
    if (rc != HALDA_OK) {
        delete P;
        return rc;
    }
    c->handles.push_back(P);
    *plan = P;
    return HALDA_OK;
}

int halda_fleets_plan_launch(void *plan, void *stream) {
    FleetsPlan *P = static_cast<FleetsPlan *>(plan);
    if (!P) return fail(HALDA_E_ARG, "NULL plan");
    if (!P->c) return fail(HALDA_E_ARG, "halda_fleets_plan_launch: the plan's context was freed");
    if (P->F.n_fleets <= 0) return HALDA_OK;
    Ctx *c = P->c;
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess || cur != c->device) HIP_TRY(hipSetDevice(c->device));
    if (P->gen != c->path_gen) {  // halda_set_fleets_path since: plan the context's current path
        const int rc = replan(P);
        if (rc != HALDA_OK) return rc;
    }
    if (!P->fused)
        return halda_solve_fleets(c, &P->model, &P->F, P->ks.data(), int32_t(P->ks.size()), &P->out, stream);
    return run_sweep(c, P->p, stream ? static_cast<hipStream_t>(stream) : c->stream);
}

int halda_fleets_plan_launch_many(void *const *plans, int32_t n_plans, void *const *streams, int32_t n_streams,
                                  int64_t first, int32_t steps) {
    if (!plans || !streams || n_plans <= 0 || n_streams <= 0 || steps < 0 || first < 0)
        return fail(HALDA_E_ARG, "halda_fleets_plan_launch_many: NULL arrays or bad counts");
    for (int32_t t = 0; t < steps; ++t) {
        const int64_t i = first + t;
        const int rc = halda_fleets_plan_launch(plans[i % n_plans], streams[i % n_streams]);
        if (rc != HALDA_OK) return rc;
    }
    return HALDA_OK;
}

void halda_fleets_plan_free(void *plan) {
    FleetsPlan *P = static_cast<FleetsPlan *>(plan);
    if (!P) return;
    if (P->c) P->c->detach(P);
    delete P;
}

}  // extern "C"

// ---- groups: `steps` batches over resident tables in one launch (halda_sweep_steps_kernel)
namespace {
struct FleetsGroup : CtxHandle {
    std::vector<FleetsPlan> plans;  // copies: the group does not depend on the caller's plan handles
    bool persistent = false;        // every plan a register (or k-slot) sweep of one shape: one launch
    bool kslot = false;             // ... the k-slot form (halda_sweep_kslot_steps_kernel + gated tables)
    int gen = 0;                    // the context's path_gen when the group was checked
    SweepArgs A;                    // the first plan's arguments (shape, model, k list)
    StepsDesc *desc = nullptr;      // device copy of the plans' tables / results
    uint8_t *fflag = nullptr;       // k-slot form: per (plan, fleet) hand-back flags
    int *hb = nullptr;              // ... the launch's hand-back flag
    int64_t lds = 0;                // ... the k-slot launch's LDS (the plan's)
};

bool same_model(const halda_model &a, const halda_model &b) { return std::memcmp(&a, &b, sizeof a) == 0; }

// Whether the group's plans can run as one steps launch, and its descriptors if so.
int group_check(FleetsGroup *G) {
    Ctx *c = G->c;
    G->gen = c->path_gen;
    G->persistent = false;
    for (FleetsPlan &P : G->plans) {
        if (P.gen != c->path_gen) {
            const int rc = replan(&P);
            if (rc != HALDA_OK) return rc;
        }
    }
    const FleetsPlan &P0 = G->plans[0];
    const bool reg = P0.fused && P0.p.kind == kRegAlone && P0.p.A.uM > 0 && P0.p.A.uM <= kK1MaxM && !P0.p.A.k1dp;
    const bool ksl = P0.fused && P0.p.kind == kKslotGated;
    bool ok = (reg || ksl) && !(P0.p.A.outs & kOutXC) && !P0.p.A.x_off;
    for (const FleetsPlan &P : G->plans) {
        ok = ok && P.fused && P.p.kind == P0.p.kind && P.F.n_fleets == P0.F.n_fleets && P.p.A.uM == P0.p.A.uM &&
             P.F.min_devices == P0.F.min_devices && P.F.max_devices == P0.F.max_devices &&
             P.p.A.outs == P0.p.A.outs && P.ks == P0.ks && same_model(P.model, P0.model) && !P.p.A.x_off &&
             P.p.lds == P0.p.lds && P.p.slice == P0.p.slice && P.p.grid2 == P0.p.grid2 &&
             P.p.block1 == P0.p.block1 && std::memcmp(&P.p.SA, &P0.p.SA, sizeof(SlotArgs)) == 0;
    }
    if (!ok) return HALDA_OK;
    std::vector<StepsDesc> h(G->plans.size());
    for (size_t i = 0; i < h.size(); ++i) {
        const FleetsPlan &P = G->plans[i];
        h[i].F = P.F;
        h[i].out = FleetOut(P.out);
        int64_t base = 0;  // dev_off[0] of the table (device memory, read once here)
        HIP_TRY(hipMemcpy(&base, P.F.dev_off, sizeof base, hipMemcpyDeviceToHost));
        h[i].base = base;
        // the steps kernel indexes the table's arrays with 32-bit byte offsets (load_fields32)
        if (reg && (base < 0 || base + int64_t(P.F.n_fleets) * P0.p.A.uM > (int64_t(1) << 29))) return HALDA_OK;
    }
    if (!G->desc) HIP_TRY(hipMalloc(&G->desc, sizeof(StepsDesc) * h.size()));
    HIP_TRY(hipMemcpy(G->desc, h.data(), sizeof(StepsDesc) * h.size(), hipMemcpyHostToDevice));
    G->A = P0.p.A;
    G->kslot = ksl;
    if (ksl) {
        G->lds = P0.p.lds;
        HIP_TRY(Ctx::ensure_lds(reinterpret_cast<const void *>(halda_sweep_kslot_steps_kernel), G->lds));
        HIP_TRY(Ctx::ensure_lds(reinterpret_cast<const void *>(halda_sweep_tables_steps_kernel), P0.p.slice));
        const size_t nfl = h.size() * size_t(P0.F.n_fleets);
        if (!G->fflag) HIP_TRY(hipMalloc(&G->fflag, std::max<size_t>(nfl, 1)));
        if (!G->hb) HIP_TRY(hipMalloc(&G->hb, sizeof(int)));
        HIP_TRY(hipMemset(G->fflag, 0, std::max<size_t>(nfl, 1)));
        HIP_TRY(hipMemset(G->hb, 0, sizeof(int)));
    }
    G->persistent = true;
    return HALDA_OK;
}
}  // namespace

extern "C" {

int halda_fleets_group_create(void *const *plans, int32_t n_plans, void **group, int32_t *persistent) {
    if (!plans || n_plans <= 0 || !group) return fail(HALDA_E_ARG, "halda_fleets_group_create: NULL arrays or n_plans <= 0");
    Ctx *c = nullptr;
    for (int32_t i = 0; i < n_plans; ++i) {
        const FleetsPlan *P = static_cast<const FleetsPlan *>(plans[i]);
        if (!P || !P->c) return fail(HALDA_E_ARG, "halda_fleets_group_create: NULL plan or freed context");
        if (c && P->c != c) return fail(HALDA_E_ARG, "halda_fleets_group_create: plans of different contexts");
        c = P->c;
    }
    HIP_TRY(hipSetDevice(c->device));
    FleetsGroup *G = new FleetsGroup();
    G->c = c;
    for (int32_t i = 0; i < n_plans; ++i) G->plans.push_back(*static_cast<const FleetsPlan *>(plans[i]));
    for (FleetsPlan &P : G->plans) P.c = c;
    const int rc = group_check(G);
    if (rc != HALDA_OK) {
        if (G->desc) (void)hipFree(G->desc);
        if (G->fflag) (void)hipFree(G->fflag);
        if (G->hb) (void)hipFree(G->hb);
        delete G;
        return rc;
    }
    c->handles.push_back(G);
    *group = G;
    if (persistent) *persistent = G->persistent ? 1 : 0;
    return HALDA_OK;
}

int halda_fleets_group_launch(void *group, int64_t first, int32_t steps, void *stream) {
    FleetsGroup *G = static_cast<FleetsGroup *>(group);
    if (!G) return fail(HALDA_E_ARG, "NULL group");
    if (!G->c) return fail(HALDA_E_ARG, "halda_fleets_group_launch: the group's context was freed");
    if (steps < 0 || first < 0) return fail(HALDA_E_ARG, "halda_fleets_group_launch: steps and first must be >= 0");
    Ctx *c = G->c;
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess || cur != c->device) HIP_TRY(hipSetDevice(c->device));
    if (G->gen != c->path_gen) {
        const int rc = group_check(G);
        if (rc != HALDA_OK) return rc;
    }
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->stream;
    const int64_t n = int64_t(G->plans.size());
    if (steps == 0 || G->plans[0].F.n_fleets <= 0) return HALDA_OK;
    if (!G->persistent) {  // batch by batch, each its own launch(es), in order on the one stream
        for (int32_t t = 0; t < steps; ++t) {
            FleetsPlan &P = G->plans[size_t((first + t) % n)];
            const int rc = P.fused ? run_sweep(c, P.p, s)
                                   : halda_solve_fleets(c, &P.model, &P.F, P.ks.data(), int32_t(P.ks.size()), &P.out, s);
            if (rc != HALDA_OK) return rc;
        }
        return HALDA_OK;
    }
    StepsArgs SG;
    SG.desc = G->desc;
    SG.n_desc = int(n);
    SG.first = int(first % n);
    SG.steps = steps;
    SG.fflag = G->fflag;
    c->fleet_timed = false;
    c->have_lowered = false;
    const int nf = G->plans[0].F.n_fleets;
    if (c->timing) HIP_TRY(hipEventRecord(c->evf0, s));
    if (G->kslot) {
        const SweepPlan &p = G->plans[0].p;
        SweepArgs A = G->A;
        A.fflag = nullptr;  // per batch: SG.fflag
        A.hb_flag = G->hb;
        A.launch_id = ++c->launch_id;
        A.want = 0;
        if (steps > 65535) return fail(HALDA_E_ARG, "halda_fleets_group_launch: more than 65,535 k-slot steps");
        // one workgroup per (batch, group of four fleets): the dispatcher's order is the items' order
        const unsigned ng = unsigned((nf + 64 / kSegLanes - 1) / (64 / kSegLanes));
        HIP_TRY(Ctx::ensure_lds(reinterpret_cast<const void *>(halda_sweep_kslot_steps_kernel), G->lds));
        hipLaunchKernelGGL(halda_sweep_kslot_steps_kernel, dim3(ng, unsigned(steps)), dim3(p.block1), size_t(G->lds), s,
                           A, p.SA, SG);
        HIP_TRY(hipGetLastError());
        if (c->timing) HIP_TRY(hipEventRecord(c->evfm, s));
        A.want = 1;  // the fleets flagged above, gated on the launch's hand-back flag
        HIP_TRY(Ctx::ensure_lds(reinterpret_cast<const void *>(halda_sweep_tables_steps_kernel), p.slice));
        hipLaunchKernelGGL(halda_sweep_tables_steps_kernel, dim3(p.grid2, unsigned(std::min<int64_t>(steps, n))),
                           dim3(64), size_t(p.slice), s, A, SG);
        HIP_TRY(hipGetLastError());
    } else {
        // one wave per (batch, fleet) item: grid (fleet blocks, steps)
        if (steps > 65535) return fail(HALDA_E_ARG, "halda_fleets_group_launch: more than 65,535 steps");
        hipLaunchKernelGGL(halda_sweep_steps_kernel,
                           dim3(unsigned((nf + kSweepWavesPerBlock - 1) / kSweepWavesPerBlock), unsigned(steps)),
                           dim3(64 * kSweepWavesPerBlock), 0, s, G->A, SG);
        HIP_TRY(hipGetLastError());
    }
    if (c->timing) {
        HIP_TRY(hipEventRecord(c->evf1, s));
        c->fleet_timed = true;
    }
    c->fleet_two = G->kslot;
    c->fleet_reg_alone = !G->kslot;
    c->fleet_seg = false;
    c->fleet_kslot = G->kslot;
    c->last_fleet_fused = true;
    return HALDA_OK;
}

void halda_fleets_group_free(void *group) {
    FleetsGroup *G = static_cast<FleetsGroup *>(group);
    if (!G) return;
    if (G->c) {
        (void)hipSetDevice(G->c->device);
        G->c->detach(G);
    }
    if (G->desc) (void)hipFree(G->desc);
    if (G->fflag) (void)hipFree(G->fflag);
    if (G->hb) (void)hipFree(G->hb);
    delete G;
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
        c->pinned_dev = nullptr;
        c->pinned_bytes = 0;
        // fine-grained (coherent): the resident wave reads and writes it between host accesses without a
        // kernel boundary in between
        HIP_TRY(hipHostMalloc(&c->pinned, off, hipHostMallocMapped | hipHostMallocCoherent));
        c->pinned_bytes = off;
    }
    char *pin = static_cast<char *>(c->pinned);
    const bool zc = off <= kZeroCopyBytes && !c->host_copy;
    // every array in halda_host_alloc blocks (the batch API's workspaces): DMA straight from / to them
    bool direct = !zc;
    if (direct) {
        const double *fa[16] = {fh->scpu_b1, fh->sgpu_b1, fh->T_cpu, fh->T_gpu, fh->t_kvcpy_cpu, fh->t_kvcpy_gpu,
                                fh->t_ram2vram, fh->t_vram2ram, fh->t_comm, fh->s_disk, fh->d_avail_ram, fh->c_cpu,
                                fh->c_gpu, fh->d_avail_cuda, fh->d_avail_metal, fh->swap};
        for (int a = 0; a < 16 && direct; ++a) direct = fa[a] && in_host_block(fa[a], 8 * nd);
        direct = direct && in_host_block(fh->dev_off, 8 * (nf + 1)) && fh->os_class && fh->flags &&
                 in_host_block(fh->os_class, nd) && in_host_block(fh->flags, nd) &&
                 in_host_block(out_h->x_off, xsel ? 8 * size_t(nf) * n_k : 0) &&
                 in_host_block(out_h->best_k, 4 * nf) && in_host_block(out_h->obj_value, 8 * nf) &&
                 in_host_block(out_h->w, 4 * nd) && in_host_block(out_h->n, 4 * nd) &&
                 in_host_block(out_h->obj_by_k, 8 * nf * n_k) && in_host_block(out_h->status, 4 * nf * n_k) &&
                 in_host_block(out_h->x, 8 * xs) && in_host_block(out_h->c, 8 * xs);
    }
    auto up = [&](size_t o, const void *src, size_t bytes) {
        if (direct) return hipMemcpyAsync(static_cast<char *>(c->scratch) + o, src, bytes, hipMemcpyHostToDevice, s);
        std::memcpy(pin + o, src, bytes);
        return hipSuccess;
    };
    halda_fleets d = *fh;
    HIP_TRY(up(o_doff, fh->dev_off, 8 * (nf + 1)));
    HIP_TRY(up(o_cls, fh->os_class, nd));
    HIP_TRY(up(o_fl, fh->flags, nd));
    const double *f64[10] = {fh->scpu_b1, fh->sgpu_b1, fh->T_cpu, fh->T_gpu, fh->t_kvcpy_cpu,
                             fh->t_kvcpy_gpu, fh->t_ram2vram, fh->t_vram2ram, fh->t_comm, fh->s_disk};
    const double *b64[6] = {fh->d_avail_ram, fh->c_cpu, fh->c_gpu, fh->d_avail_cuda, fh->d_avail_metal, fh->swap};
    for (int a = 0; a < 10; ++a) {
        if (!f64[a] || !fh->os_class || !fh->flags) return fail(HALDA_E_ARG, "halda_fleets has a NULL array");
        HIP_TRY(up(o_f64 + 8 * nd * a, f64[a], 8 * nd));
    }
    for (int a = 0; a < 6; ++a) {
        if (!b64[a]) return fail(HALDA_E_ARG, "halda_fleets has a NULL array");
        HIP_TRY(up(o_i64 + 8 * nd * a, b64[a], 8 * nd));
    }
    // small calls (a single halda_solve: ~8 KB in, ~70 KB out) skip both copies: the kernels read the
    // table from and write the results to the pinned buffer itself, across PCIe, and the host polls
    // the completion event instead of sleeping in a stream synchronisation
    if (xsel) HIP_TRY(up(o_xoff, out_h->x_off, 8 * size_t(nf) * n_k));
    if (zc) {
        if (!c->pinned_dev) HIP_TRY(hipHostGetDevicePointer(&c->pinned_dev, c->pinned, 0));
        base = static_cast<char *>(c->pinned_dev);
    } else if (!direct) {
        HIP_TRY(hipMemcpyAsync(base, pin, o_bk, hipMemcpyHostToDevice, s));  // the table (and x_off)
    }
    auto F64 = [&](int a) { return reinterpret_cast<const double *>(base + o_f64 + 8 * nd * a); };
    auto I64 = [&](int a) { return reinterpret_cast<const double *>(base + o_i64 + 8 * nd * a); };
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
    bool resident = false;
    if (zc && nf == 1 && c->fleets_fused && c->resident && n_k <= 64) {
        // one fleet, the register-only plan: the resident wave, no launch
        const int rc0 = check_fleets_args(model, &d, ks, n_k, &r);
        if (rc0 != HALDA_OK) {
            c->x_zero = true;
            return rc0;
        }
        SweepPlan *p = nullptr;
        bool retry = false;
        int rc1 = cached_plan(c, *model, d, ks, n_k, r, &p);
        if (rc1 == HALDA_OK) rc1 = resident_sweep(c, *p, &resident, &retry);
        c->x_zero = rc1 != HALDA_OK || retry ? true : c->x_zero;
        if (rc1 != HALDA_OK) return rc1;
        if (retry) return halda_solve_fleets_host(ctx, model, fh, ks, n_k, out_h);  // on a fresh pinned buffer
    }
    const int rc = resident ? HALDA_OK : halda_solve_fleets(ctx, model, &d, ks, n_k, &r, s);
    c->x_zero = true;
    if (rc != HALDA_OK) return rc;
    if (resident) {
        // the results are in the pinned buffer (ack was published after them)
    } else if (zc) {
        HIP_TRY(hipEventRecord(c->ev_host, s));
        hipError_t q;
        while ((q = hipEventQuery(c->ev_host)) == hipErrorNotReady) {
        }
        HIP_TRY(q);
    } else if (direct) {
        auto dn = [&](void *dst, size_t o, size_t bytes) {
            return dst ? hipMemcpyAsync(dst, base + o, bytes, hipMemcpyDeviceToHost, s) : hipSuccess;
        };
        HIP_TRY(dn(out_h->best_k, o_bk, 4 * nf));
        HIP_TRY(dn(out_h->obj_value, o_obj, 8 * nf));
        HIP_TRY(dn(out_h->w, o_w, 4 * nd));
        HIP_TRY(dn(out_h->n, o_n, 4 * nd));
        HIP_TRY(dn(out_h->obj_by_k, o_obk, 8 * nf * n_k));
        HIP_TRY(dn(out_h->status, o_st, 4 * nf * n_k));
        HIP_TRY(dn(out_h->x, o_x, 8 * xs));
        HIP_TRY(dn(out_h->c, o_c, 8 * xs));
        HIP_TRY(hipStreamSynchronize(s));
        return HALDA_OK;
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
    ncclComm_t cm = static_cast<ncclComm_t>(comm);
    int world = 0, rank = 0;
    NCCL_TRY(ncclCommCount(cm, &world));
    NCCL_TRY(ncclCommUserRank(cm, &rank));
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->stream;
    std::vector<ShardRank> R(1);
    R[0].rank = rank;
    R[0].o = *out;
    // the ranks' all-reduces over RCCL, on this rank's results, in the step order of shard_steps
    auto ar = [&](ShardField fld, size_t count) -> int {
        const halda_fleet_result &o = R[0].o;
        switch (fld) {
            case kShObj: NCCL_TRY(ncclAllReduce(o.obj_value, o.obj_value, count, ncclFloat64, ncclMin, cm, s)); break;
            case kShBestK: NCCL_TRY(ncclAllReduce(o.best_k, o.best_k, count, ncclInt32, ncclMin, cm, s)); break;
            case kShGroupStart: NCCL_TRY(ncclGroupStart()); break;
            case kShW: NCCL_TRY(ncclAllReduce(o.w, o.w, count, ncclInt32, ncclSum, cm, s)); break;
            case kShN: NCCL_TRY(ncclAllReduce(o.n, o.n, count, ncclInt32, ncclSum, cm, s)); break;
            case kShObk: NCCL_TRY(ncclAllReduce(o.obj_by_k, o.obj_by_k, count, ncclFloat64, ncclMin, cm, s)); break;
            case kShSt: NCCL_TRY(ncclAllReduce(o.status, o.status, count, ncclInt32, ncclMax, cm, s)); break;
            case kShGroupEnd: NCCL_TRY(ncclGroupEnd()); break;
        }
        return HALDA_OK;
    };
    return shard_steps(c, *model, *fleets, ks, n_k, world, R, s, ar);
}

int halda_solve_fleets_sharded_emulated(void *ctx, int32_t world, int32_t report_rank, const halda_model *model,
                                        const halda_fleets *fleets, const int32_t *ks, int32_t n_k,
                                        halda_fleet_result *out, void *stream) {
    Ctx *c = static_cast<Ctx *>(ctx);
    if (!c || !model || !fleets || !ks || !out) return fail(HALDA_E_ARG, "NULL argument");
    if (world < 1 || world > kEmuMaxWorld || report_rank < 0 || report_rank >= world)
        return fail(HALDA_E_ARG, "halda_solve_fleets_sharded_emulated: need 1 <= world <= 16, 0 <= report_rank < world");
    if (!out->best_k || !out->obj_value || !out->w || !out->n) return fail(HALDA_E_ARG, "halda_fleet_result: NULL");
    if (out->x || out->c) return fail(HALDA_E_ARG, "halda_solve_fleets_sharded: x / c are not gathered (pass NULL)");
    if (fleets->n_fleets > 0) {  // n_k, ks and the arrays before any size is computed or HIP call made
        const int rc = check_fleets_args(model, fleets, ks, n_k, out);
        if (rc != HALDA_OK) return rc;
    }
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->stream;
    const int64_t nf = fleets->n_fleets;
    if (nf <= 0) return HALDA_OK;
    int64_t nd = 0;
    {
        const int rc = shard_device_count(*fleets, s, &nd);
        if (rc != HALDA_OK) return rc;
    }
    // every virtual rank but report_rank gets its own result arrays (the caller's are report_rank's)
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off += (bytes + 255) & ~size_t(255); return o; };
    std::vector<size_t> o_bk(world), o_obj(world), o_w(world), o_n(world), o_obk(world), o_st(world);
    for (int r = 0; r < world; ++r) {
        o_bk[r] = take(4 * nf);
        o_obj[r] = take(8 * nf);
        o_w[r] = take(4 * size_t(nd));
        o_n[r] = take(4 * size_t(nd));
        o_obk[r] = take(8 * size_t(nf) * n_k);
        o_st[r] = take(4 * size_t(nf) * n_k);
    }
    if (off > c->emu_bytes) {
        if (c->emu) HIP_TRY(hipFree(c->emu));
        c->emu = nullptr;
        c->emu_bytes = 0;
        HIP_TRY(hipMalloc(&c->emu, off));
        c->emu_bytes = off;
    }
    char *base = static_cast<char *>(c->emu);
    std::vector<ShardRank> R(static_cast<size_t>(world));
    for (int r = 0; r < world; ++r) {
        R[size_t(r)].rank = r;
        halda_fleet_result &o = R[size_t(r)].o;
        if (r == report_rank) {
            o = *out;
            continue;
        }
        o = {};
        o.best_k = reinterpret_cast<int32_t *>(base + o_bk[r]);
        o.obj_value = reinterpret_cast<double *>(base + o_obj[r]);
        o.w = reinterpret_cast<int32_t *>(base + o_w[r]);
        o.n = reinterpret_cast<int32_t *>(base + o_n[r]);
        o.obj_by_k = out->obj_by_k ? reinterpret_cast<double *>(base + o_obk[r]) : nullptr;
        o.status = out->status ? reinterpret_cast<int32_t *>(base + o_st[r]) : nullptr;
    }
    // each all-reduce as one device kernel over the virtual ranks' buffers (in place, every rank's copy
    // gets the reduced value), in the step order of shard_steps
    auto ar = [&](ShardField fld, size_t count) -> int {
        if (fld == kShGroupStart || fld == kShGroupEnd) return HALDA_OK;
        EmuReduce E = {};
        E.world = world;
        E.count = int64_t(count);
        E.field = int(fld);
        for (int r = 0; r < world; ++r) {
            const halda_fleet_result &o = R[size_t(r)].o;
            E.p[r] = fld == kShObj ? static_cast<void *>(o.obj_value) : fld == kShBestK ? static_cast<void *>(o.best_k)
                   : fld == kShW ? static_cast<void *>(o.w) : fld == kShN ? static_cast<void *>(o.n)
                   : fld == kShObk ? static_cast<void *>(o.obj_by_k) : static_cast<void *>(o.status);
        }
        if (count == 0) return HALDA_OK;
        hipLaunchKernelGGL(halda_emu_allreduce_kernel, dim3(unsigned((count + 255) / 256)), dim3(256), 0, s, E);
        HIP_TRY(hipGetLastError());
        return HALDA_OK;
    };
    return shard_steps(c, *model, *fleets, ks, n_k, world, R, s, ar);
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
