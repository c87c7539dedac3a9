// C ABI of the engine (include/riptide_amd.h): host-buffer drop-ins for
// riptide.libcpp and the device-resident batched periodogram.
#include "riptide_amd.h"
#ifdef RT_TEST_HOOKS
#include "riptide_amd_test.h"
#endif

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "kernels.hpp"
#include "plan.hpp"

using namespace rt;

namespace {

thread_local std::string g_err;
thread_local int g_device = 0;

int fail(int code, const std::string& msg)
{
    g_err = msg;
    return code;
}

struct HipError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

inline void ck(hipError_t e, const char* what)
{
    if (e != hipSuccess) throw HipError(std::string(what) + ": " + hipGetErrorString(e));
}

// Exception barrier for every entry point.
template <class F>
int guarded(F&& f)
{
    try {
        return f();
    } catch (const std::invalid_argument& e) {
        return fail(RT_EINVAL, e.what());
    } catch (const HipError& e) {
        return fail(RT_EHIP, e.what());
    } catch (const std::exception& e) {
        return fail(RT_EINTERNAL, e.what());
    } catch (...) {
        return fail(RT_EINTERNAL, "unknown error");
    }
}

// ---- per-device context for host-buffer calls: stream + grow-only buffers
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    void* get(size_t n)
    {
        if (n > bytes) {
            if (p) (void)hipFree(p);
            p = nullptr;
            bytes = 0;
            ck(hipMalloc(&p, std::max<size_t>(n, 256)), "hipMalloc");
            bytes = std::max<size_t>(n, 256);
        }
        return p;
    }
};

struct Context {
    int device = -1;
    hipStream_t stream = nullptr;
    DevBuf buf[6];
};

std::mutex g_mu;
std::vector<Context*> g_ctx;

Context& context()
{
    ck(hipSetDevice(g_device), "hipSetDevice");
    if ((int)g_ctx.size() <= g_device) g_ctx.resize(g_device + 1, nullptr);
    if (!g_ctx[g_device]) {
        Context* c = new Context();
        c->device = g_device;
        ck(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking), "hipStreamCreate");
        g_ctx[g_device] = c;
    }
    return *g_ctx[g_device];
}

template <class T>
T* dev(Context& c, int slot, size_t count)
{
    return (T*)c.buf[slot].get(count * sizeof(T));
}

void h2d(void* d, const void* h, size_t bytes, hipStream_t s)
{
    if (bytes) ck(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s), "hipMemcpyAsync H2D");
}

void d2h(void* h, const void* d, size_t bytes, hipStream_t s)
{
    if (bytes) ck(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s), "hipMemcpyAsync D2H");
}

void sync(hipStream_t s) { ck(hipStreamSynchronize(s), "hipStreamSynchronize"); }

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Per-trial scratch budget (floats per ping/pong buffer) of one transform group.
// Tuning knob for experiments: RIPTIDE_AMD_SCRATCH_MFLOATS (millions of floats).
uint64_t scratch_budget_floats()
{
    if (const char* e = std::getenv("RIPTIDE_AMD_SCRATCH_MFLOATS")) {
        const double v = std::atof(e);
        if (v > 0) return (uint64_t)(v * 1e6);
    }
    return 96ull << 20;   // 384 MiB per ping/pong buffer and trial: ~94 launches per cfg2 plan (sweep_schedule.py)
}

// Scratch banks of a periodogram plan: 2 (RIPTIDE_AMD_COSCHED=1) runs its
// transform groups co-scheduled on two streams (run_cone_launches)
uint32_t cosched_banks()
{
    const char* e = std::getenv("RIPTIDE_AMD_COSCHED");
    return e && e[0] == '1' ? 2u : 1u;
}

// ---- profiling of cone / downsample launches
struct ProfRec {
    hipEvent_t a, b;
    double alg, moved;
};
// One profiler per process, shared by every host thread (one per GPU is the
// supported model): `mu` guards the record lists and the event pool.
struct Profiler {
    std::mutex mu;
    std::atomic<bool> on{false};
    std::vector<ProfRec> rec[2];
    std::vector<hipEvent_t> pool;
    hipEvent_t ev()
    {
        if (!pool.empty()) {
            hipEvent_t e = pool.back();
            pool.pop_back();
            return e;
        }
        hipEvent_t e;
        ck(hipEventCreate(&e), "hipEventCreate");
        return e;
    }
} g_prof;

#ifdef RT_TEST_HOOKS
// test builds only (libriptide_amd_testhooks.so): plans uploaded while set
// carry one corrupt unit (tests toggle it through rt_test_corrupt_next_plans)
std::atomic<int> g_test_corrupt{0};
#endif

// ---- a compiled plan resident on one device
// A side stream and events for co-scheduled pass sequences (run_cone_launches),
// taken by one call at a time from the plan's pool.
struct SideSet {
    hipStream_t s2 = nullptr;
    hipEvent_t err_join = nullptr;   // error path: joins s2 back into the caller's stream
    std::vector<hipEvent_t> ev;
};

// Makes `device` current for a scope and restores the caller's device on
// exit: the side streams and events of a plan belong to the plan's device,
// whatever device the calling thread has current.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int device)
    {
        int cur = 0;
        ck(hipGetDevice(&cur), "hipGetDevice");
        if (cur != device) {
            ck(hipSetDevice(device), "hipSetDevice");
            prev = cur;
        }
    }
    ~DeviceGuard()
    {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
};

struct DevicePlan {
    ExecPlan ex;
    UnitDesc* d_units = nullptr;
    uint32_t* d_blob = nullptr;     // tile-unit metadata (build_tile_blob)
    int device = 0;
    mutable std::mutex side_mu;
    mutable std::vector<std::unique_ptr<SideSet>> side_all;
    mutable std::vector<SideSet*> side_free;
    ~DevicePlan()
    {
        if (d_units) (void)hipFree(d_units);
        if (d_blob) (void)hipFree(d_blob);
        for (auto& ss : side_all) {
            for (hipEvent_t e : ss->ev) (void)hipEventDestroy(e);
            if (ss->err_join) (void)hipEventDestroy(ss->err_join);
            if (ss->s2) (void)hipStreamDestroy(ss->s2);
        }
    }
    // A side stream and `events` events on the plan's device (created there
    // whatever the calling thread's current device is).
    SideSet* take_side(size_t events) const
    {
        std::lock_guard<std::mutex> lk(side_mu);
        DeviceGuard dg(device);
        SideSet* ss;
        if (!side_free.empty()) {
            ss = side_free.back();
            side_free.pop_back();
        } else {
            side_all.push_back(std::make_unique<SideSet>());
            ss = side_all.back().get();
            ck(hipStreamCreateWithFlags(&ss->s2, hipStreamNonBlocking), "hipStreamCreate");
            ck(hipEventCreateWithFlags(&ss->err_join, hipEventDisableTiming), "hipEventCreate");
        }
        while (ss->ev.size() < events) {
            hipEvent_t e;
            ck(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
            ss->ev.push_back(e);
        }
        return ss;
    }
    void give_side(SideSet* ss) const
    {
        std::lock_guard<std::mutex> lk(side_mu);
        side_free.push_back(ss);
    }
    void upload()
    {
        ck(hipGetDevice(&device), "hipGetDevice");
        std::vector<UnitDesc> u(ex.items.size());
        for (size_t i = 0; i < u.size(); ++i) {
            const ConeItem& it = ex.items[i];
            const FfaXform& X = ex.xf[it.xform];
            UnitDesc d{};
            d.node_start = it.node_start;
            d.node_size = it.node_size;
            d.s0 = it.s0;
            d.s1 = it.s1;
            d.p = X.p;
            d.m = X.m;
            d.rows_eval = X.rows_eval;
            d.stdnoise = X.stdnoise;
            d.src_off = X.src_off;
            d.buf_off = X.buf_off;
            d.snr_row = X.snr_row;
            d.levels = it.levels;
            d.mode = it.mode;
            d.src = it.src;
            d.dst = it.dst;
            d.pad = it.pad;
            if (it.pad != kNoBlob) {
                const uint32_t* h = ex.blob.data() + it.pad;
                d.nruns = h[kHdrRuns];
                d.entries = h[kHdrEntries];
                d.nb = h[kHdrBottom];
                d.slot_words = h[kHdrSlotWords];
                d.run_off = h[kHdrRunOff];
                d.fill_chunks = h[kHdrFill];
                d.zero_row = h[kHdrZero];
            }
            u[i] = d;
        }
#ifdef RT_TEST_HOOKS
        // test-only hook (rt_test_corrupt_next_plans): give the first
        // whole-node unit more merge levels than any kernel instance runs,
        // after the host validation, so the kernel's own check refuses it and
        // sets the error flag (exercises rt_plan_check)
        if (g_test_corrupt.load(std::memory_order_relaxed))
            for (UnitDesc& d : u)
                if (d.mode == kModeWhole) {
                    d.levels = kMaxLevels + 1;
                    break;
                }
#endif
        ck(hipMalloc(&d_blob, std::max<size_t>(4, ex.blob.size()) * sizeof(uint32_t)), "hipMalloc");
        if (!ex.blob.empty())
            ck(hipMemcpy(d_blob, ex.blob.data(), ex.blob.size() * sizeof(uint32_t), hipMemcpyHostToDevice),
               "upload blob");
        ck(hipMalloc(&d_units, std::max<size_t>(1, u.size()) * sizeof(UnitDesc)), "hipMalloc");
        if (!u.empty())
            ck(hipMemcpy(d_units, u.data(), u.size() * sizeof(UnitDesc), hipMemcpyHostToDevice), "upload units");
    }
};

// Per-phase cycle counters of the cone kernel (RT_STAMPS diagnostic builds).
unsigned long long* g_stamps = nullptr;
uint64_t g_stamp_units = 0;      // unit records written since the last reset
std::vector<uint64_t> g_stamp_launch;   // first record of each launch since the last reset

// Run all cone launches of an exec plan.
// One cone launch of a plan on stream s (profiling: HIP events around it
// unless `prof_each` is off).
void cone_launch(const DevicePlan& P, const Launch& L, ConeArgs a, uint32_t batch, hipStream_t s, bool prof_each)
{
    a.items = P.d_units + L.first;
    a.num_items = L.count;
    const uint64_t units = (uint64_t)L.count * batch;   // one workgroup per (item, trial)
    if (L.count > 0x7FFFFFFFu || batch > 65535u) throw std::invalid_argument("too many cone work units in one launch");
    // diagnostic builds: this launch's unit records follow the previous ones
    a.stamps = nullptr;
    if (g_stamps) {
        std::lock_guard<std::mutex> lk(g_prof.mu);
        if (g_stamp_units + units <= kTimelineCap) {
            a.stamps = g_stamps + g_stamp_units * kStampRecWords;
            g_stamp_launch.push_back(g_stamp_units);
            g_stamp_units += units;
        }
    }
    ProfRec r{};
    const bool prof = g_prof.on && prof_each;
    if (prof) {
        {
            std::lock_guard<std::mutex> lk(g_prof.mu);
            r.a = g_prof.ev();
            r.b = g_prof.ev();
        }
        r.alg = L.alg_bytes * batch;
        r.moved = L.moved_bytes * batch;
        ck(hipEventRecord(r.a, s), "hipEventRecord");
    }
    ck(launch_cone(a, L.smax, L.rw, L.wide_snr != 0, L.snr != 0, s), "cone_kernel");
    if (prof) {
        ck(hipEventRecord(r.b, s), "hipEventRecord");
        std::lock_guard<std::mutex> lk(g_prof.mu);
        g_prof.rec[0].push_back(r);
    }
}

// A side set taken from a plan's pool for one launch sequence: returned to
// the pool on every exit.  While `forked`, launches may be queued on the side
// stream that the caller's stream has not joined; an exception then joins
// them back (so the caller cannot reuse or free the workspace while the side
// stream still writes it) before the set goes back to the pool.
struct SideLease {
    const DevicePlan& P;
    SideSet* ss;
    hipStream_t s;
    bool forked = false;
    SideLease(const DevicePlan& plan, size_t events, hipStream_t caller) : P(plan), ss(plan.take_side(events)), s(caller) {}
    ~SideLease()
    {
        if (forked) {
            DeviceGuard dg(P.device);
            if (hipEventRecord(ss->err_join, ss->s2) != hipSuccess || hipStreamWaitEvent(s, ss->err_join, 0) != hipSuccess)
                (void)hipStreamSynchronize(ss->s2);
        }
        P.give_side(ss);
    }
    SideLease(const SideLease&) = delete;
    SideLease& operator=(const SideLease&) = delete;
};

// RIPTIDE_AMD_SINGLE_STREAM=1: every cone launch of a plan on the caller's
// stream, in plan order, one profiling record per launch (per-launch A/B
// measurements and the parity test of the two-stream scheduling).
bool single_stream_forced()
{
    const char* e = std::getenv("RIPTIDE_AMD_SINGLE_STREAM");
    return e && e[0] == '1';
}

// Trials per cone workgroup (ConeArgs::trials_per_wg): one workgroup runs an
// item for up to this many trials of the batch, its record, blob and roll
// table loaded once.  RIPTIDE_AMD_TRIALS_PER_WG overrides the default.
uint32_t cone_trials_per_wg()
{
    if (const char* e = std::getenv("RIPTIDE_AMD_TRIALS_PER_WG")) {
        const long v = std::strtol(e, nullptr, 10);
        if (v >= 1 && v <= 65535) return (uint32_t)v;
    }
    return kConeTrialsPerWg;
}

// Run all cone launches of an exec plan.  A plan with two scratch banks
// (ExecPlan::banks) runs its transform groups co-scheduled on two streams:
// group g on stream g mod 2, its merge-only launches starting once group g - 1
// has finished its own merge-only launches -- so group g's merge-only passes
// (latency / LDS bound) share the CUs with group g - 1's final passes (VALU
// bound: the fused S/N).  Profiling then records one event pair around the
// whole sequence (launches overlap) with their summed algorithmic bytes.
void run_cone_launches(const DevicePlan& P, ConeArgs a, uint32_t batch, hipStream_t s)
{
    a.batch = batch;
    a.trials_per_wg = cone_trials_per_wg();
    a.flags = kConeDefaultFeatures;
    if (const char* e = std::getenv("RIPTIDE_AMD_CONE_FLAGS")) a.flags = (uint32_t)std::strtoul(e, nullptr, 0);
    // the 4/5-slot instances have no dense per-level path since round 5: the
    // fused two-level merge is their only merge, so the bit cannot be turned
    // off (an A/B value without it would leave their units unwritten)
    a.flags |= kConeFuse2;
    a.blob = P.d_blob;
    const std::vector<Launch>& Ls = P.ex.launches;
    DeviceGuard dg(P.device);
    const bool single = single_stream_forced();
    if (single || P.ex.banks < 2 || P.ex.groups < 2) {
        bool multi = false;
        for (const Launch& L : Ls) multi = multi || L.smax != Ls.front().smax;
        if (!multi || single) {
            for (const Launch& L : Ls) cone_launch(P, L, a, batch, s, true);
            return;
        }
        // slot-width buckets on two streams: within a transform group the
        // launches of different slot widths belong to disjoint transforms
        // (independent pass chains), so the group's main bucket (most cells)
        // runs on s and the others on a side stream, joined at the group's
        // end (the next group reuses the scratch buffers).  Each chain's
        // launch drains fill with the other's units: cone ms per trial cfg2
        // 7.092 -> 7.072, cfg3 1.795 -> 1.776, cfg1 0.274 -> 0.260
        // (profiles/r04r_ab_*_bucketstreams.log); the cone time is then one
        // profiling record from the fork to the join.
        const uint32_t G = std::max<uint32_t>(P.ex.groups, 1);
        SideLease lease(P, 2 * (size_t)G, s);
        SideSet* const ss = lease.ss;
        ProfRec r{};
        const bool prof = g_prof.on;
        if (prof) {
            {
                std::lock_guard<std::mutex> lk(g_prof.mu);
                r.a = g_prof.ev();
                r.b = g_prof.ev();
            }
            for (const Launch& L : Ls) {
                r.alg += L.alg_bytes * batch;
                r.moved += L.moved_bytes * batch;
            }
            ck(hipEventRecord(r.a, s), "hipEventRecord");
        }
        size_t li = 0;
        for (uint32_t g = 0; g < G && li < Ls.size(); ++g) {
            size_t l1 = li;
            std::map<uint32_t, uint64_t> cells;
            while (l1 < Ls.size() && Ls[l1].group == Ls[li].group) cells[Ls[l1].smax] += Ls[l1].cells, ++l1;
            uint32_t mainb = Ls[li].smax;
            for (const auto& kv : cells) if (kv.second > cells[mainb]) mainb = kv.first;
            ck(hipEventRecord(ss->ev[2 * g], s), "hipEventRecord");
            ck(hipStreamWaitEvent(ss->s2, ss->ev[2 * g], 0), "hipStreamWaitEvent");
            lease.forked = true;
            for (; li < l1; ++li) cone_launch(P, Ls[li], a, batch, Ls[li].smax == mainb ? s : ss->s2, false);
            ck(hipEventRecord(ss->ev[2 * g + 1], ss->s2), "hipEventRecord");
            ck(hipStreamWaitEvent(s, ss->ev[2 * g + 1], 0), "hipStreamWaitEvent");
            lease.forked = false;
        }
        if (li != Ls.size()) throw std::runtime_error("cone launches out of group order");
        if (prof) {
            ck(hipEventRecord(r.b, s), "hipEventRecord");
            std::lock_guard<std::mutex> lk(g_prof.mu);
            g_prof.rec[0].push_back(r);
        }
        return;
    }
    const uint32_t G = P.ex.groups;
    SideLease lease(P, 2 + (size_t)G, s);
    SideSet* const ss = lease.ss;
    ProfRec r{};
    const bool prof = g_prof.on;
    if (prof) {
        {
            std::lock_guard<std::mutex> lk(g_prof.mu);
            r.a = g_prof.ev();
            r.b = g_prof.ev();
        }
        for (const Launch& L : Ls) {
            r.alg += L.alg_bytes * batch;
            r.moved += L.moved_bytes * batch;
        }
        ck(hipEventRecord(r.a, s), "hipEventRecord");
    }
    hipEvent_t fork = ss->ev[0], join = ss->ev[1];
    ck(hipEventRecord(fork, s), "hipEventRecord");
    ck(hipStreamWaitEvent(ss->s2, fork, 0), "hipStreamWaitEvent");
    lease.forked = true;
    size_t li = 0;
    for (uint32_t g = 0; g < G; ++g) {
        hipStream_t st = (g & 1u) ? ss->s2 : s;
        if (g >= 1) ck(hipStreamWaitEvent(st, ss->ev[2 + g - 1], 0), "hipStreamWaitEvent");
        while (li < Ls.size() && Ls[li].group == g && !Ls[li].snr) cone_launch(P, Ls[li++], a, batch, st, false);
        ck(hipEventRecord(ss->ev[2 + g], st), "hipEventRecord");
        while (li < Ls.size() && Ls[li].group == g) cone_launch(P, Ls[li++], a, batch, st, false);
    }
    if (li != Ls.size()) throw std::runtime_error("cone launches out of group order");
    ck(hipEventRecord(join, ss->s2), "hipEventRecord");
    ck(hipStreamWaitEvent(s, join, 0), "hipStreamWaitEvent");
    lease.forked = false;
    if (prof) {
        ck(hipEventRecord(r.b, s), "hipEventRecord");
        std::lock_guard<std::mutex> lk(g_prof.mu);
        g_prof.rec[0].push_back(r);
    }
}

// Single-transform FFA (ffa2 / benchmark_ffa2): in (device) -> out (device).
// d_flag: device int the cone kernel sets if a unit breaks its budget (the
// caller checks it after synchronising).  A plan built here is freed only
// after the stream has drained; a cached plan lives in the caller.
void ffa_device(const float* d_in, size_t rows, size_t cols, float* d_out, float* d_tmp, int* d_flag, hipStream_t s,
                DevicePlan* cached = nullptr)
{
    if (!rows || !cols) return;
    if (lds_row_capacity((uint32_t)cols) >= 3 && (uint64_t)rows * cols * 4u < kMaxBlockBytes) {
        DevicePlan local;
        DevicePlan& P = cached ? *cached : local;
        if (!cached || P.ex.launches.empty()) {
            FfaXform X{};
            X.p = (uint32_t)cols;
            X.m = (uint32_t)rows;
            build_exec_plan({X}, false, 0, ~0ull, P.ex);
            P.upload();
        }
        ConeArgs a{};
        a.leaves = d_in;
        a.ping = d_out;
        a.pong = d_tmp;
        a.error_flag = d_flag;
        run_cone_launches(P, a, 1, s);
        if (!cached) sync(s);   // `local` (and its unit table) is freed on return
        return;
    }
    // rows too wide for LDS: per-depth global-memory passes
    int depth = 0;
    while ((1ull << depth) < rows) ++depth;
    std::vector<std::vector<uint2>> levels(depth + 1);
    levels[0].push_back(make_uint2(0, (uint32_t)rows));
    for (int d = 0; d < depth; ++d)
        for (const uint2& n : levels[d]) {
            if (n.y <= 1) { levels[d + 1].push_back(n); continue; }
            const uint32_t h = n.y >> 1;
            levels[d + 1].push_back(make_uint2(n.x, h));
            levels[d + 1].push_back(make_uint2(n.x + h, n.y - h));
        }
    uint2* d_nodes = nullptr;
    ck(hipMalloc(&d_nodes, std::max<size_t>(1, rows) * sizeof(uint2)), "hipMalloc");
    const float* src = d_in;
    for (int d = depth - 1; d >= 0; --d) {
        float* dst = ((d % 2) == 0) ? d_out : d_tmp;
        ck(hipMemcpyAsync(d_nodes, levels[d].data(), levels[d].size() * sizeof(uint2), hipMemcpyHostToDevice, s),
           "nodes");
        ck(launch_ffa_level(src, dst, d_nodes, (uint32_t)levels[d].size(), (uint32_t)rows, (uint32_t)cols, s),
           "ffa_level");
        ck(hipStreamSynchronize(s), "sync");
        src = dst;
    }
    if (depth == 0) ck(hipMemcpyAsync(d_out, d_in, rows * cols * 4, hipMemcpyDeviceToDevice, s), "copy");
    ck(hipStreamSynchronize(s), "sync");
    (void)hipFree(d_nodes);
}

void check_widths(const uint64_t* w, size_t nw, size_t bins)
{
    for (size_t i = 0; i < nw; ++i)
        if (!(w[i] > 0 && w[i] < bins)) throw std::invalid_argument("trial widths must be all > 0 and < columns");
}

}  // namespace

// ---------------------------------------------------------------------------
// periodogram plan
// ---------------------------------------------------------------------------
struct rt_plan {
    PgramPlan pg;
    DevicePlan dp;
    std::vector<uint32_t> widths;
    uint32_t* d_widths = nullptr;
    std::vector<DsRung> rungs;
    DsRung* d_rungs = nullptr;
    uint32_t ds_blocks = 0;
    // kLadderPerRung / kLadderFused (every rung fits the fused ladder's
    // margin) / kLadderHybrid (the rungs that fit take the fused kernel, the
    // wider ones the per-rung kernel: rungs_w, first_block within the subset)
    int ds_mode = 0;
    std::vector<DsRung> rungs_f, rungs_w;
    DsRung* d_rungs_f = nullptr;
    DsRung* d_rungs_w = nullptr;
    uint32_t ds_blocks_w = 0;
    int* d_flag = nullptr;   // sticky device error flag of the cone kernel (rt_plan_check reads and clears it)
    ~rt_plan()
    {
        if (d_rungs) (void)hipFree(d_rungs);
        if (d_rungs_f) (void)hipFree(d_rungs_f);
        if (d_rungs_w) (void)hipFree(d_rungs_w);
        if (d_widths) (void)hipFree(d_widths);
        if (d_flag) (void)hipFree(d_flag);
    }
};

namespace {

// The fused ladder (downsample_fused_kernel) indexes samples and outputs in
// 32 bits and stages up to kDsFusedMargin floats past each span: series of 2^29
// samples or more, rungs whose window (ceil(f) + 2) exceeds the margin, and
// more rungs than its per-block table take the per-rung kernel (64-bit
// indices) instead.
constexpr uint64_t kDsFusedMaxSize = 1ull << 29;
constexpr int kLadderPerRung = 0, kLadderFused = 1, kLadderHybrid = 2;

bool rung_fusable(const DsRung& d) { return d.identity || std::ceil(d.f) + 2.0 <= (double)kDsFusedMargin; }

// The ladder's kernels for a plan's rungs: every rung in the fused kernel;
// or, when some rungs' windows exceed its margin (cfg5's long range: factors
// up to ~1950), the others in the fused kernel and those in the per-rung
// kernel (hybrid, `f` / `w` the two subsets, w's first_block renumbered);
// or all per-rung (series of 2^29 samples or more: 32-bit indices; more
// fusable rungs than the fused kernel's per-block table).
int ladder_split(size_t size, const std::vector<DsRung>& rungs, std::vector<DsRung>* f, std::vector<DsRung>* w)
{
    if ((uint64_t)size >= kDsFusedMaxSize) return kLadderPerRung;
    std::vector<DsRung> a, b;
    uint32_t blocks = 0;
    for (const DsRung& d : rungs) {
        if (rung_fusable(d)) {
            a.push_back(d);
        } else {
            DsRung e = d;
            e.first_block = blocks;
            blocks += (uint32_t)((e.n + e.per_block - 1) / e.per_block);
            b.push_back(e);
        }
    }
    if (a.empty() || a.size() > kDsMaxRungs || ds_fused_margin(a.data(), a.size()) == 0) return kLadderPerRung;
    if (f) *f = a;
    if (w) *w = b;
    return b.empty() ? kLadderFused : kLadderHybrid;
}

// The rungs of a periodogram that feed at least one transform, in the
// ladder kernels' form.
std::vector<DsRung> used_rungs(const PgramPlan& pg)
{
    std::vector<bool> used(pg.rungs.size(), false);
    for (const Step& s : pg.steps)
        if (s.rows_eval) used[s.rung] = true;
    std::vector<DsRung> out;
    uint32_t blocks = 0;
    for (size_t r = 0; r < pg.rungs.size(); ++r) {
        if (!used[r]) continue;
        const Rung& R = pg.rungs[r];
        DsRung d{};
        d.f = R.f;
        d.n = R.n;
        d.out_off = R.leaf_off;
        d.first_block = blocks;
        d.identity = R.f == 1.0;
        ds_configure(d);
        blocks += (uint32_t)((R.n + d.per_block - 1) / d.per_block);
        out.push_back(d);
    }
    return out;
}

rt_plan* make_plan(size_t size, double tsamp, const uint64_t* widths, size_t nw, double pmin, double pmax,
                   size_t bmin, size_t bmax)
{
    PgramParams prm;
    prm.size = size;
    prm.tsamp = tsamp;
    prm.pmin = pmin;
    prm.pmax = pmax;
    prm.bmin = bmin;
    prm.bmax = bmax;
    const std::string msg = check_pgram_args(prm);
    if (!msg.empty()) throw std::invalid_argument(msg);
    if (nw > (size_t)kMaxWidths) throw std::invalid_argument("at most 32 trial widths are supported");
    check_widths(widths, nw, bmin);
    if (lds_row_capacity((uint32_t)bmax) < 3) throw std::invalid_argument("bins_max too large for the LDS FFA engine");
    auto* P = new rt_plan();
    try {
        build_pgram_plan(prm, P->pg);
        P->widths.assign(widths, widths + nw);
        ck(hipMalloc(&P->d_widths, std::max<size_t>(1, nw) * sizeof(uint32_t)), "hipMalloc");
        if (nw)
            ck(hipMemcpy(P->d_widths, P->widths.data(), nw * sizeof(uint32_t), hipMemcpyHostToDevice), "upload widths");
        std::vector<FfaXform> xf;
        for (const Step& s : P->pg.steps) {
            if (!s.rows_eval) continue;   // nothing of this transform reaches the output
            FfaXform X{};
            X.p = s.bins;
            X.m = s.rows;
            X.rows_eval = s.rows_eval;
            X.rung = s.rung;
            X.src_off = P->pg.rungs[s.rung].leaf_off;
            X.snr_row = s.out_row;
            X.stdnoise = s.stdnoise;
            xf.push_back(X);
        }
        // scratch budget per ping/pong buffer and trial (scratch_budget_floats)
        const uint32_t wmax = P->widths.empty() ? 0u : *std::max_element(P->widths.begin(), P->widths.end());
        build_exec_plan(xf, true, (uint32_t)nw, scratch_budget_floats(), P->dp.ex, wmax, cosched_banks());
        P->dp.upload();
        ck(hipMalloc(&P->d_flag, sizeof(int)), "hipMalloc");
        ck(hipMemset(P->d_flag, 0, sizeof(int)), "hipMemset");
        // downsample ladder over the rungs that feed at least one transform
        P->rungs = used_rungs(P->pg);
        P->ds_blocks = 0;
        for (const DsRung& d : P->rungs) P->ds_blocks += (uint32_t)((d.n + d.per_block - 1) / d.per_block);
        P->ds_mode = std::getenv("RIPTIDE_AMD_PER_RUNG_LADDER")
                         ? kLadderPerRung
                         : ladder_split(prm.size, P->rungs, &P->rungs_f, &P->rungs_w);
        for (const DsRung& d : P->rungs_w) P->ds_blocks_w += (uint32_t)((d.n + d.per_block - 1) / d.per_block);
        auto upload = [](DsRung*& dst, const std::vector<DsRung>& src) {
            ck(hipMalloc(&dst, std::max<size_t>(1, src.size()) * sizeof(DsRung)), "hipMalloc");
            if (!src.empty())
                ck(hipMemcpy(dst, src.data(), src.size() * sizeof(DsRung), hipMemcpyHostToDevice), "upload rungs");
        };
        upload(P->d_rungs, P->rungs);
        if (P->ds_mode != kLadderPerRung) upload(P->d_rungs_f, P->rungs_f);
        if (P->ds_mode == kLadderHybrid) upload(P->d_rungs_w, P->rungs_w);
    } catch (...) {
        delete P;
        throw;
    }
    return P;
}

size_t plan_ws_bytes(const rt_plan* P, size_t batch)
{
    size_t b = align_up(P->pg.leaf_floats * 4 * batch, 256);
    b += 2 * align_up(P->dp.ex.scratch_floats * 4 * batch, 256);
    b += 256;   // slack
    return b;
}

// Workspace layout: [leaves | ping | pong]
struct PlanWs {
    float* leaves;
    float* ping;
    float* pong;
};

PlanWs plan_ws(const rt_plan* P, size_t batch, void* ws, size_t ws_bytes)
{
    if (ws_bytes < plan_ws_bytes(P, batch)) throw std::invalid_argument("workspace too small");
    char* w = (char*)ws;
    PlanWs o;
    o.leaves = (float*)w;
    w += align_up(P->pg.leaf_floats * 4 * batch, 256);
    o.ping = (float*)w;
    w += align_up(P->dp.ex.scratch_floats * 4 * batch, 256);
    o.pong = (float*)w;
    return o;
}

// The downsampling ladder of a batch into the workspace's leaf buffer.
void run_ladder(const rt_plan* P, const float* d_data, size_t batch, size_t data_stride, void* ws, size_t ws_bytes,
                hipStream_t s)
{
    float* const leaves = plan_ws(P, batch, ws, ws_bytes).leaves;
    ProfRec r{};
    const bool prof = g_prof.on;
    if (prof) {
        {
            std::lock_guard<std::mutex> lk(g_prof.mu);
            r.a = g_prof.ev();
            r.b = g_prof.ev();
        }
        ck(hipEventRecord(r.a, s), "hipEventRecord");
    }
    if (P->ds_mode != kLadderPerRung)
        ck(launch_downsample_fused(d_data, P->pg.prm.size, data_stride, P->d_rungs_f, (uint32_t)P->rungs_f.size(),
                                   ds_fused_margin(P->rungs_f.data(), P->rungs_f.size()), leaves, P->pg.leaf_floats,
                                   (uint32_t)batch, s),
           "downsample_fused");
    if (P->ds_mode == kLadderHybrid)
        ck(launch_downsample_ladder(d_data, P->pg.prm.size, data_stride, P->d_rungs_w, (uint32_t)P->rungs_w.size(),
                                    P->ds_blocks_w, leaves, P->pg.leaf_floats, (uint32_t)batch, s),
           "downsample_ladder");
    if (P->ds_mode == kLadderPerRung)
        ck(launch_downsample_ladder(d_data, P->pg.prm.size, data_stride, P->d_rungs, (uint32_t)P->rungs.size(),
                                    P->ds_blocks, leaves, P->pg.leaf_floats, (uint32_t)batch, s),
           "downsample_ladder");
    if (prof) {
        ck(hipEventRecord(r.b, s), "hipEventRecord");
        // fused: the series is read once for its rungs; per-rung: once per rung
        double bytes = P->ds_mode != kLadderPerRung ? 4.0 * P->pg.prm.size : 0.0;
        for (const DsRung& d : P->rungs) {
            const bool fused = P->ds_mode == kLadderFused || (P->ds_mode == kLadderHybrid && rung_fusable(d));
            bytes += 4.0 * (double)d.n + (fused ? 0.0 : (d.identity ? 4.0 * d.n : 4.0 * P->pg.prm.size));
        }
        r.alg = r.moved = bytes * batch;
        std::lock_guard<std::mutex> lk(g_prof.mu);
        g_prof.rec[1].push_back(r);
    }
}

// The FFA passes + fused S/N of a batch whose leaf buffer run_ladder filled.
void run_passes(const rt_plan* P, size_t batch, float* d_snrs, size_t snr_stride, void* ws, size_t ws_bytes,
                hipStream_t s)
{
    const PlanWs W = plan_ws(P, batch, ws, ws_bytes);
    float* const leaves = W.leaves;
    float* const ping = W.ping;
    float* const pong = W.pong;
    ConeArgs a{};
    a.num_widths = (uint32_t)P->widths.size();
    a.widths = P->d_widths;
    a.leaves = leaves;
    a.leaves_stride = P->pg.leaf_floats;
    a.ping = ping;
    a.pong = pong;
    a.buf_stride = P->dp.ex.scratch_floats;
    a.snr = d_snrs;
    a.snr_stride = snr_stride;
    a.error_flag = P->d_flag;
    run_cone_launches(P->dp, a, (uint32_t)batch, s);
}

void run_periodogram(const rt_plan* P, const float* d_data, size_t batch, size_t data_stride, float* d_snrs,
                     size_t snr_stride, void* ws, size_t ws_bytes, hipStream_t s)
{
    run_ladder(P, d_data, batch, data_stride, ws, ws_bytes, s);
    run_passes(P, batch, d_snrs, snr_stride, ws, ws_bytes, s);
}

// Dereddening + normalisation (device).  Workspace layout: [lores | rmed | partials]
struct DeredGeom {
    size_t sf = 1, n_lo = 0, rmed_w = 0;
    size_t lores_floats = 0, rmed_floats = 0, partial_doubles = 0;
    size_t slope_doubles = 0;   // np.interp segment slopes (sf > 1)
};
constexpr uint32_t kNormBlocks = 512;

DeredGeom dered_geom(size_t size, size_t ws, size_t minpts, size_t batch, bool deredden)
{
    DeredGeom g;
    if (deredden) {
        if (!(minpts % 2)) throw std::invalid_argument("min_points must be an odd number");
        const double q = (double)ws / (double)minpts;
        g.sf = (size_t)std::max(1.0, q);
        if (g.sf == 1) {
            g.n_lo = size;
            g.rmed_w = ws;
        } else {
            g.n_lo = size / g.sf;
            g.rmed_w = minpts;
            g.lores_floats = align_up(g.n_lo * batch, 64);
            g.slope_doubles = align_up(g.n_lo * batch, 32);
        }
        if (!(g.rmed_w % 2)) throw std::invalid_argument("width must be an odd number");
        if (!(g.rmed_w < g.n_lo)) throw std::invalid_argument("width must be < size");
        g.rmed_floats = align_up(g.n_lo * batch, 64);
    }
    // the unfused normalisation's partials, or the fused one's (two per
    // dereddening block: launch_deredden_normalise), then 2 * batch stats
    g.partial_doubles = std::max<size_t>((size_t)kNormBlocks, deredden ? 2 * dered_norm_blocks(size) : 0) * batch +
                        2 * batch + 8;
    return g;
}

size_t dered_ws_bytes(const DeredGeom& g)
{
    return (g.lores_floats + g.rmed_floats) * 4 + (g.slope_doubles + g.partial_doubles) * 8 + 256;
}

void run_deredden_normalise(const float* d_in, size_t size, size_t batch, size_t in_stride, const DeredGeom& g,
                            bool deredden, bool normalise, float* d_out, size_t out_stride, void* ws, hipStream_t s)
{
    float* lores = (float*)ws;
    float* rmed = lores + g.lores_floats;
    double* slopes = (double*)align_up((size_t)(rmed + g.rmed_floats), 256);
    double* partials = slopes + g.slope_doubles;
    const float* cur = d_in;
    size_t cur_stride = in_stride;
    const bool fused = deredden && normalise && g.sf > 1 &&
                       dered_norm_fusable(d_in, size, g.n_lo, (uint32_t)g.sf, d_out, in_stride, out_stride);
    if (deredden) {
        const float* rin = d_in;
        size_t rstride = in_stride;
        if (g.sf > 1) {
            ck(launch_scrunch(d_in, g.n_lo, (uint32_t)g.sf, lores, in_stride, g.n_lo, (uint32_t)batch, s), "scrunch");
            rin = lores;
            rstride = g.n_lo;
        }
        ck(launch_running_median(rin, g.n_lo, (uint32_t)g.rmed_w, rmed, rstride, g.n_lo, (uint32_t)batch, s),
           "running_median");
        if (fused) {
            const size_t np = 2 * dered_norm_blocks(size) * batch;
            ck(launch_deredden_normalise(d_in, size, rmed, g.n_lo, (uint32_t)g.sf, d_out, in_stride, g.n_lo,
                                         out_stride, (uint32_t)batch, s, slopes, partials, partials + np),
               "deredden_normalise");
            return;
        }
        ck(launch_deredden_subtract(d_in, size, rmed, g.n_lo, (uint32_t)g.sf, d_out, in_stride, g.n_lo, out_stride,
                                    (uint32_t)batch, s, g.slope_doubles ? slopes : nullptr),
           "deredden_subtract");
        cur = d_out;
        cur_stride = out_stride;
    }
    if (normalise) {
        ck(launch_normalise(cur, size, d_out, partials, kNormBlocks, cur_stride, out_stride, (uint32_t)batch, s),
           "normalise");
    } else if (!deredden && cur != d_out) {
        for (size_t b = 0; b < batch; ++b)
            ck(hipMemcpyAsync(d_out + b * out_stride, d_in + b * in_stride, size * 4, hipMemcpyDeviceToDevice, s),
               "copy");
    }
}

}  // namespace

// ---------------------------------------------------------------------------
// entry points
// ---------------------------------------------------------------------------
extern "C" {

const char* rt_last_error(void) { return g_err.c_str(); }

const char* rt_version(void) { return "riptide_amd 0.1.0 (gfx950)"; }

int rt_set_device(int device)
{
    return guarded([&] {
        ck(hipSetDevice(device), "hipSetDevice");
        g_device = device;
        return RT_OK;
    });
}

int rt_rollback(const float* x, size_t size, size_t shift, float* out)
{
    return guarded([&] {
        if (!size) return RT_OK;
        std::lock_guard<std::mutex> lk(g_mu);
        Context& c = context();
        float* dx = dev<float>(c, 0, size);
        float* dz = dev<float>(c, 1, size);
        h2d(dx, x, size * 4, c.stream);
        ck(launch_rollback(dx, size, shift, nullptr, dz, c.stream), "rollback");
        d2h(out, dz, size * 4, c.stream);
        sync(c.stream);
        return RT_OK;
    });
}

int rt_fused_rollback_add(const float* x, const float* y, size_t size, size_t shift, float* out)
{
    return guarded([&] {
        if (!size) return RT_OK;
        std::lock_guard<std::mutex> lk(g_mu);
        Context& c = context();
        float* dx = dev<float>(c, 0, size);
        float* dy = dev<float>(c, 1, size);
        float* dz = dev<float>(c, 2, size);
        h2d(dx, x, size * 4, c.stream);
        h2d(dy, y, size * 4, c.stream);
        ck(launch_rollback(dx, size, shift, dy, dz, c.stream), "fused_rollback_add");
        d2h(out, dz, size * 4, c.stream);
        sync(c.stream);
        return RT_OK;
    });
}

int rt_circular_prefix_sum(const float* x, size_t size, size_t nsum, float* out)
{
    return guarded([&] {
        if (!nsum) return RT_OK;
        if (!size) throw std::invalid_argument("circular_prefix_sum of an empty array");
        std::lock_guard<std::mutex> lk(g_mu);
        Context& c = context();
        float* dx = dev<float>(c, 0, size);
        float* dz = dev<float>(c, 1, nsum + 1);
        h2d(dx, x, size * 4, c.stream);
        ck(launch_circular_prefix_sum(dx, size, nsum, dz, c.stream), "circular_prefix_sum");
        d2h(out, dz, nsum * 4, c.stream);
        sync(c.stream);
        return RT_OK;
    });
}

int rt_ffa2(const float* in, size_t rows, size_t cols, float* out)
{
    return guarded([&] {
        if (!rows || !cols) return RT_OK;
        if (rows > 0x7FFFFFFFull || rows * cols > (1ull << 40)) throw std::invalid_argument("ffa2 input too large");
        std::lock_guard<std::mutex> lk(g_mu);
        Context& c = context();
        const size_t n = rows * cols;
        float* dx = dev<float>(c, 0, n);
        float* dz = dev<float>(c, 1, n);
        float* dt = dev<float>(c, 2, n);
        int* flag = dev<int>(c, 5, 1);
        ck(hipMemsetAsync(flag, 0, sizeof(int), c.stream), "hipMemsetAsync");
        h2d(dx, in, n * 4, c.stream);
        ffa_device(dx, rows, cols, dz, dt, flag, c.stream);
        int hflag = 0;
        d2h(&hflag, flag, sizeof hflag, c.stream);
        d2h(out, dz, n * 4, c.stream);
        sync(c.stream);
        if (hflag) throw std::runtime_error("cone kernel: work item exceeded the LDS budget");
        return RT_OK;
    });
}

int rt_benchmark_ffa2(size_t rows, size_t cols, size_t loops, double* seconds)
{
    return guarded([&] {
        *seconds = 0;
        if (!rows || !cols || !loops) return RT_OK;
        std::lock_guard<std::mutex> lk(g_mu);
        Context& c = context();
        const size_t n = rows * cols;
        float* dx = dev<float>(c, 0, n);
        float* dz = dev<float>(c, 1, n);
        float* dt = dev<float>(c, 2, n);
        int* flag = dev<int>(c, 5, 1);
        ck(hipMemsetAsync(dx, 0, n * 4, c.stream), "memset");
        ck(hipMemsetAsync(flag, 0, sizeof(int), c.stream), "hipMemsetAsync");
        DevicePlan P;
        ffa_device(dx, rows, cols, dz, dt, flag, c.stream, &P);   // warm-up + plan
        hipEvent_t a, b;
        ck(hipEventCreate(&a), "event");
        ck(hipEventCreate(&b), "event");
        ck(hipEventRecord(a, c.stream), "record");
        for (size_t i = 0; i < loops; ++i) ffa_device(dx, rows, cols, dz, dt, flag, c.stream, &P);
        ck(hipEventRecord(b, c.stream), "record");
        ck(hipEventSynchronize(b), "sync");
        float ms = 0;
        ck(hipEventElapsedTime(&ms, a, b), "elapsed");
        (void)hipEventDestroy(a);
        (void)hipEventDestroy(b);
        int hflag = 0;
        ck(hipMemcpy(&hflag, flag, sizeof hflag, hipMemcpyDeviceToHost), "flag");
        if (hflag) throw std::runtime_error("cone kernel: work item exceeded the LDS budget");
        *seconds = ms * 1e-3 / (double)loops;
        return RT_OK;
    });
}

int rt_snr2(const float* x, size_t rows, size_t cols, const uint64_t* widths, size_t nw, float stdnoise, float* out)
{
    return guarded([&] {
        if (!(stdnoise > 0)) throw std::invalid_argument("stdnoise must be > 0");
        check_widths(widths, nw, cols);
        if (!rows || !nw) return RT_OK;
        std::lock_guard<std::mutex> lk(g_mu);
        Context& c = context();
        const size_t n = rows * cols;
        float* dx = dev<float>(c, 0, n);
        float* dc = dev<float>(c, 1, n + rows);
        uint32_t* dw = dev<uint32_t>(c, 2, nw);
        float* dz = dev<float>(c, 3, rows * nw);
        std::vector<uint32_t> w32(widths, widths + nw);
        h2d(dx, x, n * 4, c.stream);
        h2d(dw, w32.data(), nw * 4, c.stream);
        ck(launch_snr_rows(dx, rows, (uint32_t)cols, dw, (uint32_t)nw, stdnoise, dc, dz, c.stream), "snr");
        d2h(out, dz, rows * nw * 4, c.stream);
        sync(c.stream);
        return RT_OK;
    });
}

int rt_snr1(const float* x, size_t size, const uint64_t* widths, size_t nw, float stdnoise, float* out)
{
    return rt_snr2(x, 1, size, widths, nw, stdnoise, out);
}

size_t rt_downsampled_size(size_t size, double f) { return downsampled_size(size, f); }

int rt_downsample(const float* x, size_t size, double f, float* out)
{
    return guarded([&] {
        // downsample.hpp:11-16
        if (!((f > 1.0) & (f <= (double)size)))
            throw std::invalid_argument("Downsampling factor must verify: 1 < f <= size");
        const size_t n = downsampled_size(size, f);
        std::lock_guard<std::mutex> lk(g_mu);
        Context& c = context();
        float* dx = dev<float>(c, 0, size);
        float* dz = dev<float>(c, 1, n);
        DsRung* dr = dev<DsRung>(c, 2, 1);
        DsRung r{};
        r.f = f;
        r.n = n;
        r.first_block = 0;
        ds_configure(r);
        h2d(dx, x, size * 4, c.stream);
        h2d(dr, &r, sizeof r, c.stream);
        ck(launch_downsample_ladder(dx, size, size, dr, 1, (uint32_t)((n + r.per_block - 1) / r.per_block), dz, n,
                                    1, c.stream),
           "downsample");
        d2h(out, dz, n * 4, c.stream);
        sync(c.stream);
        return RT_OK;
    });
}

int rt_downsample_rows(const float* x, size_t rows, size_t size, double f, float* out)
{
    return guarded([&] {
        if (!((f > 1.0) & (f <= (double)size)))
            throw std::invalid_argument("Downsampling factor must verify: 1 < f <= size");
        if (!rows) return RT_OK;
        if (rows > 65535) throw std::invalid_argument("at most 65535 rows per call");
        const size_t n = downsampled_size(size, f);
        std::lock_guard<std::mutex> lk(g_mu);
        Context& c = context();
        float* dx = dev<float>(c, 0, rows * size);
        float* dz = dev<float>(c, 1, rows * n);
        DsRung* dr = dev<DsRung>(c, 2, 1);
        DsRung r{};
        r.f = f;
        r.n = n;
        r.first_block = 0;
        ds_configure(r);
        h2d(dx, x, rows * size * 4, c.stream);
        h2d(dr, &r, sizeof r, c.stream);
        ck(launch_downsample_ladder(dx, size, size, dr, 1, (uint32_t)((n + r.per_block - 1) / r.per_block), dz, n,
                                    (uint32_t)rows, c.stream),
           "downsample");
        d2h(out, dz, rows * n * 4, c.stream);
        sync(c.stream);
        return RT_OK;
    });
}

int rt_periodogram_length(size_t size, double tsamp, double pmin, double pmax, size_t bmin, size_t bmax,
                          size_t* length)
{
    return guarded([&] {
        PgramParams prm;
        prm.size = size;
        prm.tsamp = tsamp;
        prm.pmin = pmin;
        prm.pmax = pmax;
        prm.bmin = bmin;
        prm.bmax = bmax;
        const std::string msg = check_pgram_args(prm);
        if (!msg.empty()) throw std::invalid_argument(msg);
        PgramPlan pg;
        build_pgram_plan(prm, pg);
        *length = pg.length;
        return RT_OK;
    });
}

int rt_periodogram(const float* data, size_t size, double tsamp, const uint64_t* widths, size_t nw, double pmin,
                   double pmax, size_t bmin, size_t bmax, double* periods, uint32_t* foldbins, float* snrs)
{
    return guarded([&] {
        std::lock_guard<std::mutex> lk(g_mu);
        Context& c = context();
        rt_plan* P = make_plan(size, tsamp, widths, nw, pmin, pmax, bmin, bmax);
        std::unique_ptr<rt_plan> hold(P);
        fill_grid(P->pg, periods, foldbins);
        const size_t L = P->pg.length;
        if (!L) return RT_OK;
        float* dx = dev<float>(c, 0, size);
        float* dz = dev<float>(c, 1, std::max<size_t>(1, L * nw));
        void* ws = c.buf[2].get(plan_ws_bytes(P, 1));
        h2d(dx, data, size * 4, c.stream);
        run_periodogram(P, dx, 1, size, dz, L * nw, ws, plan_ws_bytes(P, 1), c.stream);
        int flag = 0;
        d2h(&flag, P->d_flag, sizeof flag, c.stream);
        d2h(snrs, dz, L * nw * 4, c.stream);
        sync(c.stream);
        if (flag) throw std::runtime_error("cone kernel: work item exceeded the LDS budget");
        return RT_OK;
    });
}

int rt_running_median(const float* x, size_t size, size_t width, float* out)
{
    return guarded([&] {
        // running_median.hpp:103-107
        if (!(width % 2)) throw std::invalid_argument("width must be an odd number");
        if (!(width < size)) throw std::invalid_argument("width must be < size");
        std::lock_guard<std::mutex> lk(g_mu);
        Context& c = context();
        float* dx = dev<float>(c, 0, size);
        float* dz = dev<float>(c, 1, size);
        h2d(dx, x, size * 4, c.stream);
        ck(launch_running_median(dx, size, (uint32_t)width, dz, size, size, 1, c.stream), "running_median");
        d2h(out, dz, size * 4, c.stream);
        sync(c.stream);
        return RT_OK;
    });
}

int rt_fast_running_median(const float* x, size_t size, size_t ws, size_t minpts, double* out)
{
    return guarded([&] {
        const DeredGeom g = dered_geom(size, ws, minpts, 1, true);
        if (g.sf == 1) throw std::invalid_argument("scrunch factor is 1: use rt_running_median");
        std::lock_guard<std::mutex> lk(g_mu);
        Context& c = context();
        float* dx = dev<float>(c, 0, size);
        double* dz = dev<double>(c, 1, size);
        float* lores = dev<float>(c, 2, g.n_lo);
        float* rmed = dev<float>(c, 3, g.n_lo);
        h2d(dx, x, size * 4, c.stream);
        ck(launch_scrunch(dx, g.n_lo, (uint32_t)g.sf, lores, size, g.n_lo, 1, c.stream), "scrunch");
        ck(launch_running_median(lores, g.n_lo, (uint32_t)g.rmed_w, rmed, g.n_lo, g.n_lo, 1, c.stream),
           "running_median");
        ck(launch_interp(size, rmed, g.n_lo, (uint32_t)g.sf, dz, c.stream), "interp");
        d2h(out, dz, size * 8, c.stream);
        sync(c.stream);
        return RT_OK;
    });
}

int rt_deredden_normalise(const float* x, size_t size, size_t ws, size_t minpts, int deredden, int normalise,
                          float* out)
{
    return guarded([&] {
        const DeredGeom g = dered_geom(size, ws, minpts, 1, deredden != 0);
        std::lock_guard<std::mutex> lk(g_mu);
        Context& c = context();
        float* dx = dev<float>(c, 0, size);
        float* dz = dev<float>(c, 1, size);
        void* w = c.buf[2].get(dered_ws_bytes(g));
        h2d(dx, x, size * 4, c.stream);
        run_deredden_normalise(dx, size, 1, size, g, deredden != 0, normalise != 0, dz, size, w, c.stream);
        d2h(out, dz, size * 4, c.stream);
        sync(c.stream);
        return RT_OK;
    });
}

int rt_periodogram_grid(size_t size, double tsamp, double pmin, double pmax, size_t bmin, size_t bmax,
                        double* periods, uint32_t* foldbins)
{
    return guarded([&] {
        PgramParams prm;
        prm.size = size;
        prm.tsamp = tsamp;
        prm.pmin = pmin;
        prm.pmax = pmax;
        prm.bmin = bmin;
        prm.bmax = bmax;
        const std::string msg = check_pgram_args(prm);
        if (!msg.empty()) throw std::invalid_argument(msg);
        PgramPlan pg;
        build_pgram_plan(prm, pg);
        fill_grid(pg, periods, foldbins);
        return RT_OK;
    });
}

int rt_ffa_schedule_check(size_t rows, size_t cols, uint64_t* launches)
{
    return guarded([&] {
        if (!rows || !cols || rows > 0xFFFFFFFFull || cols > 0xFFFFFFFFull || !merge_slots((uint32_t)cols))
            throw std::invalid_argument("rt_ffa_schedule_check: bad shape");
        FfaXform X{};
        X.p = (uint32_t)cols;
        X.m = (uint32_t)rows;
        X.rows_eval = (uint32_t)rows;
        ExecPlan ex;
        build_exec_plan({X}, false, 0, ~0ull, ex);   // validates
        if (launches) *launches = ex.launches.size();
        return RT_OK;
    });
}

int rt_ladder_check(size_t size, double tsamp, double pmin, double pmax, size_t bmin, size_t bmax, int* fused,
                    uint64_t* rungs)
{
    return guarded([&] {
        PgramParams prm;
        prm.size = size;
        prm.tsamp = tsamp;
        prm.pmin = pmin;
        prm.pmax = pmax;
        prm.bmin = bmin;
        prm.bmax = bmax;
        const std::string msg = check_pgram_args(prm);
        if (!msg.empty()) throw std::invalid_argument(msg);
        PgramPlan pg;
        build_pgram_plan(prm, pg);
        const std::vector<DsRung> r = used_rungs(pg);
        if (fused) *fused = ladder_split(size, r, nullptr, nullptr);
        if (rungs) *rungs = r.size();
        return RT_OK;
    });
}

int rt_schedule_check(size_t size, double tsamp, size_t nw, double pmin, double pmax, size_t bmin, size_t bmax,
                      uint64_t* transforms, uint64_t* items, uint64_t* launches, double* alg_bytes,
                      double* moved_bytes, uint64_t* cells)
{
    return guarded([&] {
        PgramParams prm;
        prm.size = size;
        prm.tsamp = tsamp;
        prm.pmin = pmin;
        prm.pmax = pmax;
        prm.bmin = bmin;
        prm.bmax = bmax;
        const std::string msg = check_pgram_args(prm);
        if (!msg.empty()) throw std::invalid_argument(msg);
        PgramPlan pg;
        build_pgram_plan(prm, pg);
        std::vector<FfaXform> xf;
        for (const Step& s : pg.steps) {
            if (!s.rows_eval) continue;
            FfaXform X{};
            X.p = s.bins;
            X.m = s.rows;
            X.rows_eval = s.rows_eval;
            X.snr_row = s.out_row;
            xf.push_back(X);
        }
        ExecPlan ex;
        // build_exec_plan validates the schedule (validate_exec_plan: tiles
        // inside nodes, LDS / register budgets, final pass covers every row)
        build_exec_plan(xf, true, (uint32_t)nw, scratch_budget_floats(), ex, 0, cosched_banks());
        uint64_t a = 0;
        double alg = 0, mv = 0;
        for (const Launch& L : ex.launches) {
            alg += L.alg_bytes;
            mv += L.moved_bytes;
            if (L.pass == 0) a += L.cells;
        }
        *transforms = ex.xf.size();
        *items = ex.items.size();
        *launches = ex.launches.size();
        *alg_bytes = alg;
        *moved_bytes = mv;
        *cells = a;
        return RT_OK;
    });
}

int rt_plan_create(size_t size, double tsamp, const uint64_t* widths, size_t nw, double pmin, double pmax,
                   size_t bmin, size_t bmax, rt_plan** plan)
{
    return guarded([&] {
        ck(hipSetDevice(g_device), "hipSetDevice");
        *plan = make_plan(size, tsamp, widths, nw, pmin, pmax, bmin, bmax);
        return RT_OK;
    });
}

void rt_plan_destroy(rt_plan* plan) { delete plan; }

int rt_plan_shape(const rt_plan* P, size_t* length, size_t* nw)
{
    *length = P->pg.length;
    *nw = P->widths.size();
    return RT_OK;
}

int rt_plan_grid(const rt_plan* P, double* periods, uint32_t* foldbins)
{
    return guarded([&] {
        fill_grid(P->pg, periods, foldbins);
        return RT_OK;
    });
}

int rt_plan_workspace_bytes(const rt_plan* P, size_t batch, size_t* bytes)
{
    *bytes = plan_ws_bytes(P, batch);
    return RT_OK;
}

int rt_periodogram_device(const rt_plan* P, const float* d_data, size_t batch, size_t data_stride, float* d_snrs,
                          size_t snr_stride, void* ws, size_t ws_bytes, void* stream)
{
    return guarded([&] {
        if (!batch || !P->pg.length) return RT_OK;
        run_periodogram(P, d_data, batch, data_stride, d_snrs, snr_stride, ws, ws_bytes, (hipStream_t)stream);
        return RT_OK;
    });
}

int rt_periodogram_ladder_device(const rt_plan* P, const float* d_data, size_t batch, size_t data_stride, void* ws,
                                 size_t ws_bytes, void* stream)
{
    return guarded([&] {
        if (!batch || !P->pg.length) return RT_OK;
        run_ladder(P, d_data, batch, data_stride, ws, ws_bytes, (hipStream_t)stream);
        return RT_OK;
    });
}

int rt_periodogram_passes_device(const rt_plan* P, size_t batch, float* d_snrs, size_t snr_stride, void* ws,
                                 size_t ws_bytes, void* stream)
{
    return guarded([&] {
        if (!batch || !P->pg.length) return RT_OK;
        run_passes(P, batch, d_snrs, snr_stride, ws, ws_bytes, (hipStream_t)stream);
        return RT_OK;
    });
}

int rt_plan_check(const rt_plan* P, void* stream)
{
    return guarded([&] {
        hipStream_t s = (hipStream_t)stream;
        int flag = 0;
        ck(hipMemcpyAsync(&flag, P->d_flag, sizeof flag, hipMemcpyDeviceToHost, s), "hipMemcpyAsync D2H");
        ck(hipStreamSynchronize(s), "hipStreamSynchronize");
        if (flag) {
            ck(hipMemsetAsync(P->d_flag, 0, sizeof(int), s), "hipMemsetAsync");
            ck(hipStreamSynchronize(s), "hipStreamSynchronize");
            throw std::runtime_error("cone kernel: work item exceeded the LDS budget (S/N rows left unwritten)");
        }
        return RT_OK;
    });
}

int rt_deredden_workspace_bytes(size_t size, size_t ws, size_t minpts, size_t batch, size_t* bytes)
{
    return guarded([&] {
        *bytes = dered_ws_bytes(dered_geom(size, ws, minpts, batch, true));
        return RT_OK;
    });
}

int rt_deredden_normalise_device(const float* d_in, size_t size, size_t batch, size_t in_stride, size_t ws,
                                 size_t minpts, int deredden, int normalise, float* d_out, size_t out_stride,
                                 void* d_ws, size_t ws_bytes, void* stream)
{
    return guarded([&] {
        const DeredGeom g = dered_geom(size, ws, minpts, batch, deredden != 0);
        if (ws_bytes < dered_ws_bytes(g)) throw std::invalid_argument("workspace too small");
        if (deredden && d_in == d_out) throw std::invalid_argument("deredden cannot run in place");
        run_deredden_normalise(d_in, size, batch, in_stride, g, deredden != 0, normalise != 0, d_out, out_stride,
                               d_ws, (hipStream_t)stream);
        return RT_OK;
    });
}

int rt_segment_order_stats_device(const float* d_snrs, size_t batch, size_t snr_stride, size_t length,
                                  size_t num_widths, size_t nseg, size_t per_seg, const uint32_t* ranks,
                                  size_t nranks, float* d_out, void* stream)
{
    return guarded([&] {
        if (!batch || !num_widths || !nseg) return RT_OK;
        if (per_seg == 0 || nseg * per_seg > length) throw std::invalid_argument("segments exceed the periodogram");
        if (per_seg > (size_t)kMaxSegmentPoints)
            throw std::invalid_argument("segment longer than the device sort (32768 points)");
        if (!nranks || nranks > (size_t)kMaxSegmentRanks) throw std::invalid_argument("1 to 8 ranks per segment");
        for (size_t r = 0; r < nranks; ++r)
            if (ranks[r] >= per_seg) throw std::invalid_argument("rank outside the segment");
        if (batch > 65535 || num_widths > 65535 || nseg > 0x7FFFFFFFull)
            throw std::invalid_argument("segment grid too large");
        ck(launch_segment_order_stats(d_snrs, snr_stride, (uint32_t)batch, (uint32_t)num_widths, (uint32_t)nseg,
                                      (uint32_t)per_seg, ranks, (uint32_t)nranks, d_out, (hipStream_t)stream),
           "segment_order_stats");
        return RT_OK;
    });
}

int rt_threshold_select_device(const float* d_snrs, size_t batch, size_t snr_stride, size_t length,
                               size_t num_widths, const double* d_logf, const double* d_coeffs, size_t ncoef,
                               double smin, uint32_t* d_counts, uint32_t* d_idx, size_t cap, void* stream)
{
    return guarded([&] {
        if (!batch || !num_widths) return RT_OK;
        if (!ncoef || ncoef > 64) throw std::invalid_argument("1 to 64 polynomial coefficients");
        if (length > 0xFFFFFFFFull || cap > 0xFFFFFFFFull || batch > 65535 || num_widths > 65535)
            throw std::invalid_argument("threshold selection too large");
        hipStream_t s = (hipStream_t)stream;
        ck(hipMemsetAsync(d_counts, 0, batch * num_widths * sizeof(uint32_t), s), "hipMemsetAsync");
        ck(launch_threshold_select(d_snrs, snr_stride, (uint32_t)batch, (uint32_t)length, (uint32_t)num_widths, d_logf,
                                   d_coeffs, (uint32_t)ncoef, smin, d_counts, d_idx, (uint32_t)cap, s),
           "threshold_select");
        return RT_OK;
    });
}

int rt_convert_samples_device(const void* d_raw, size_t n, int is_signed, float* d_out, void* stream)
{
    return guarded([&] {
        if (n >= (1ull << 42)) throw std::invalid_argument("too many samples");
        ck(launch_convert_samples(d_raw, n, is_signed, d_out, (hipStream_t)stream), "convert_samples");
        return RT_OK;
    });
}

int rt_profile_enable(int on)
{
    g_prof.on = on != 0;
    return RT_OK;
}

int rt_profile_reset(void)
{
    return guarded([&] {
        std::lock_guard<std::mutex> lk(g_prof.mu);
        for (auto& v : g_prof.rec)
            for (auto& r : v) {
                g_prof.pool.push_back(r.a);
                g_prof.pool.push_back(r.b);
            }
        g_prof.rec[0].clear();
        g_prof.rec[1].clear();
        return RT_OK;
    });
}

int rt_profile_read(int kind, double* ms, double* alg, double* moved, uint64_t* launches)
{
    return guarded([&] {
        if (kind < 0 || kind > 1) throw std::invalid_argument("kind must be 0 or 1");
        std::lock_guard<std::mutex> lk(g_prof.mu);
        double t = 0, b = 0, mv = 0;
        for (auto& r : g_prof.rec[kind]) {
            ck(hipEventSynchronize(r.b), "hipEventSynchronize");
            float e = 0;
            ck(hipEventElapsedTime(&e, r.a, r.b), "hipEventElapsedTime");
            t += e;
            b += r.alg;
            mv += r.moved;
        }
        *ms = t;
        *alg = b;
        *moved = mv;
        *launches = g_prof.rec[kind].size();
        return RT_OK;
    });
}

int rt_diag_stamps(uint64_t* out8, int reset)
{
    return guarded([&] {
        if (!g_stamps) {
            ck(hipMalloc(&g_stamps, kTimelineCap * kStampRecWords * sizeof(unsigned long long)), "hipMalloc");
            ck(hipMemset(g_stamps, 0, kTimelineCap * kStampRecWords * sizeof(unsigned long long)), "hipMemset");
        }
        ck(hipDeviceSynchronize(), "hipDeviceSynchronize");
        for (int i = 0; i < 8; ++i) out8[i] = 0;
        std::lock_guard<std::mutex> lk(g_prof.mu);
        out8[0] = g_stamp_units;
        if (reset) {
            g_stamp_units = 0;
            g_stamp_launch.clear();
        }
        return RT_OK;
    });
}

int rt_diag_launches(uint64_t* out, uint64_t cap, uint64_t* count)
{
    return guarded([&] {
        std::lock_guard<std::mutex> lk(g_prof.mu);
        const uint64_t n = std::min<uint64_t>(g_stamp_launch.size(), cap);
        for (uint64_t i = 0; i < n; ++i) out[i] = g_stamp_launch[i];
        *count = n;
        return RT_OK;
    });
}

int rt_diag_timeline(uint64_t* out, uint64_t cap, uint64_t* count)
{
    return guarded([&] {
        *count = 0;
        if (!g_stamps) return RT_OK;
        ck(hipDeviceSynchronize(), "hipDeviceSynchronize");
        const uint64_t n = std::min<uint64_t>(std::min<uint64_t>(g_stamp_units, kTimelineCap), cap);
        *count = n;
        if (n)
            ck(hipMemcpy(out, g_stamps, n * kStampRecWords * sizeof(uint64_t), hipMemcpyDeviceToHost), "hipMemcpy");
        return RT_OK;
    });
}

int rt_plan_stats(const rt_plan* P, uint64_t* transforms, uint64_t* items, uint64_t* launches, double* alg,
                  double* moved, uint64_t* cells)
{
    *transforms = P->dp.ex.xf.size();
    *items = P->dp.ex.items.size();
    *launches = P->dp.ex.launches.size();
    double a = 0, m = 0;
    uint64_t c = 0;
    for (const Launch& L : P->dp.ex.launches) {
        a += L.alg_bytes;
        m += L.moved_bytes;
        if (L.pass == 0) c += L.cells;
    }
    *alg = a;
    *moved = m;
    *cells = c;
    return RT_OK;
}

}  // extern "C"

#ifdef RT_TEST_HOOKS
int rt_test_corrupt_next_plans(int on)
{
    g_test_corrupt.store(on ? 1 : 0, std::memory_order_relaxed);
    return RT_OK;
}
#endif
