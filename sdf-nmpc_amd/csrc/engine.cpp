// C ABI implementation (include/sdfnmpc.h): contexts, device-resident packed networks, launches.
//
// Host-side runtime only: all arithmetic of the hot path happens in sdf_mlp.hip / linearize.hip.
// There is no CPU fallback: without a HIP device every compute entry point fails with
// SDFNMPC_E_NODEVICE / SDFNMPC_E_HIP.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "../../include/sdfnmpc.h"
#include "lin_kernels.h"
#include "qp_kernels.h"
#include "ref_kernels.h"
#include "sdf_kernels.h"
#include "vae_kernels.h"

using namespace sdfn;

// ------------------------------------------------------------------------------------------------
// errors
static thread_local std::string g_err;
static int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
#define HIPCHK(expr)                                                                              \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess) return fail(SDFNMPC_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

extern "C" int sdfnmpc_abi_version(void) { return SDFNMPC_ABI_VERSION; }
// error reporting for solver.hip (same thread-local message)
extern "C" int sdfnmpc_solver_fail_(int code, const char* msg) { return fail(code, msg); }
extern "C" const char* sdfnmpc_last_error(void) { return g_err.c_str(); }

// ------------------------------------------------------------------------------------------------
// context
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    unsigned long long gen = 0;  // reallocations so far (a captured step graph holds the pointer of its time)
    hipError_t ensure(size_t n) {
        if (n <= bytes) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        ++gen;
        hipError_t e = hipMalloc(&p, n);
        if (e == hipSuccess) bytes = n;
        return e;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

struct KStat {
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
    double ms = 0.0;
    long long n = 0;
};

struct sdfnmpc_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    hipStream_t aux = nullptr;                       // low-priority side stream (fork/join per call)
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    bool lin_first = false;
    bool serial_prep = false;  // diagnostic (SDFNMPC_SERIAL_PREP=1): linearize after the SDF kernel, same stream
    int qp_kernel = SDFNMPC_QP_AUTO;  // SDFNMPC_QP_KERNEL=serial|segmented, or sdfnmpc_ctx_set_qp_kernel
    int tile_rows = 32;
    int n_cu = 0;              // compute units of the device (hipDeviceProp_t::multiProcessorCount)
    size_t lds_per_cu = 0;     // LDS bytes per CU (hipDeviceProp_t::maxSharedMemoryPerMultiProcessor)
    bool timing = false;
    DevBuf c13, sdf4, lat, out4, glat, qpw, qpst, wws;
    // host-pointer path (sdf_eval_host, the CasADi external): pinned staging, its own hoist buffer and
    // the latents it was computed for (consecutive acados calls share one latent: the hoist is reused)
    float* h_pin = nullptr;
    size_t h_pin_bytes = 0;
    DevBuf hin, hout, hc13;
    std::vector<float> h_lat;
    uint64_t h_net = 0;  // uid of the network the cached hoist belongs to
    // resident SDF server of the host path (sdf_row.hip, SdfMbox): mailbox in pinned coherent memory, its
    // own stream, the network it serves, the last request number, and whether it may still be running
    struct {
        int mode = -1;                // -1: from SDFNMPC_SDF_SERVER (default on), 0 off, 1 on
        SdfMbox* mb = nullptr;
        SdfMbox* mb_dev = nullptr;
        hipStream_t stream = nullptr;
        uint64_t net = 0;
        unsigned long long seq = 0;
        bool live = false;
        long long idle_ticks = 0, life_ticks = 0;
        double idle_s = 0.001, life_s = 0.0008;  // SDFNMPC_SDF_SERVER_IDLE_MS / _LIFE_MS
        unsigned long long epoch = 0;           // launches so far; the live server's is in `gone` once it left
        bool abandoned = false;                 // a server that would not stop: its mailbox is never reused
        double khz = 100000.0;
        std::chrono::steady_clock::time_point last{};
        double acc[4] = {0, 0, 0, 0};  // diagnostics: us staging, computing, host round trip; calls
        double ph[14] = {};            // diagnostics: us per row_eval phase
    } srv;
    std::map<std::string, KStat> stats;
    std::mutex mu;  // serialises the host-pointer path (CasADi externals may be called concurrently)
    // stage records packed by sdfnmpc_rti_prepare, consumed by the next sdfnmpc_qp_feedback
    struct {
        bool valid = false;
        int B = 0, N = 0;
        const double* xn = nullptr;  // the lin outputs they were packed from
        const void* work = nullptr;
        bool sdf_row_patch = false;  // the feedback's QP kernel copies the sdf row of C^T into them
        int ny = 0, cost_scaling = 0, lm_scaling = 0;  // the qp options the records were packed under
        double lm = 0.0;
        long long cset = 0;  // and their constraint set (cset_key)
    } prep;
};

struct ScopedDevice {
    int prev = -1;
    explicit ScopedDevice(int d) {
        (void)hipGetDevice(&prev);
        if (prev != d) (void)hipSetDevice(d);
    }
    ~ScopedDevice() {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
    }
};

// launch helper with optional HIP-event timing on the context stream
template <typename F>
static hipError_t timed(sdfnmpc_ctx* ctx, const char* name, F&& launch, hipStream_t st = nullptr) {
    if (!ctx->timing) return launch();
    if (!st) st = ctx->stream;
    hipEvent_t a, b;
    hipError_t e = hipEventCreate(&a);
    if (e != hipSuccess) return e;
    e = hipEventCreate(&b);
    if (e != hipSuccess) return e;
    (void)hipEventRecord(a, st);
    e = launch();
    (void)hipEventRecord(b, st);
    ctx->stats[name].pending.emplace_back(a, b);
    return e;
}

extern "C" int sdfnmpc_ctx_create(int device, void* stream, sdfnmpc_ctx** out) {
    if (!out) return fail(SDFNMPC_E_ARG, "out is NULL");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return fail(SDFNMPC_E_NODEVICE, "no HIP device visible: the sdfnmpc compute path has no CPU fallback");
    if (device < 0 || device >= n) return fail(SDFNMPC_E_ARG, "device index out of range");
    ScopedDevice sd(device);
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    if (std::string(prop.gcnArchName).rfind("gfx950", 0) != 0)
        return fail(SDFNMPC_E_UNSUPPORTED, std::string("built for gfx950 only, device is ") + prop.gcnArchName);
    HIPCHK(sdf_set_lds_limits());
    auto* c = new sdfnmpc_ctx();
    c->device = device;
    c->n_cu = prop.multiProcessorCount;
    c->lds_per_cu = prop.maxSharedMemoryPerMultiProcessor;
    if (stream) {
        c->stream = (hipStream_t)stream;
    } else {
        hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
        if (e != hipSuccess) {
            delete c;
            return fail(SDFNMPC_E_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(e));
        }
        c->own_stream = true;
    }
    int lo = 0, hi = 0;
    hipError_t e = hipDeviceGetStreamPriorityRange(&lo, &hi);  // lo = least urgent
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&c->aux, hipStreamNonBlocking, lo);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming);
    if (e != hipSuccess) {
        sdfnmpc_ctx_destroy(c);
        return fail(SDFNMPC_E_HIP, std::string("aux stream/events: ") + hipGetErrorString(e));
    }
    const char* lf = getenv("SDFNMPC_LIN_FIRST");
    c->lin_first = lf && *lf == '1';
    const char* sp = getenv("SDFNMPC_SERIAL_PREP");
    c->serial_prep = sp && *sp == '1';
    if (const char* qk = getenv("SDFNMPC_QP_KERNEL")) {
        if (!strcmp(qk, "serial")) c->qp_kernel = SDFNMPC_QP_SERIAL;
        else if (!strcmp(qk, "segmented")) c->qp_kernel = SDFNMPC_QP_SEGMENTED;
    }
    *out = c;
    return SDFNMPC_OK;
}

// Ask the resident SDF server to exit and wait for it, polling with a deadline (a server that stopped
// answering must not hang destroy / reconfigure while the shim's lock is held): on timeout the mailbox
// and stream are abandoned -- never freed or reused, since the server may still write to them -- and
// the host path falls back to one launch per call.  Returns false on timeout.
static void mark_abandoned(uint64_t uid);
static bool srv_stop(sdfnmpc_ctx* ctx) {
    auto& S = ctx->srv;
    if (!S.mb || S.abandoned) return !S.abandoned;
    __atomic_store_n(&S.mb->stop, 1ull, __ATOMIC_RELEASE);
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t q = hipStreamQuery(S.stream);
        if (q != hipErrorNotReady) break;
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > 2.0) {
            S.abandoned = true;
            S.live = false;
            S.mode = 0;
            mark_abandoned(S.net);  // its network is leaked, not freed under a running reader
            fail(SDFNMPC_E_HIP, "sdf server: did not stop within 2 s; abandoned (one launch per call from now on)");
            return false;
        }
        std::this_thread::yield();
    }
    __atomic_store_n(&S.mb->stop, 0ull, __ATOMIC_RELEASE);
    S.live = false;
    return true;
}

extern "C" void sdfnmpc_ctx_destroy(sdfnmpc_ctx* ctx) {
    if (!ctx) return;
    ScopedDevice sd(ctx->device);
    if (ctx->srv.mb && srv_stop(ctx)) {
        (void)hipStreamDestroy(ctx->srv.stream);
        (void)hipHostFree(ctx->srv.mb);
    }
    (void)hipStreamSynchronize(ctx->stream);
    for (auto& kv : ctx->stats)
        for (auto& ev : kv.second.pending) {
            (void)hipEventDestroy(ev.first);
            (void)hipEventDestroy(ev.second);
        }
    if (ctx->aux) {
        (void)hipStreamSynchronize(ctx->aux);
        (void)hipStreamDestroy(ctx->aux);
    }
    if (ctx->h_pin) (void)hipHostFree(ctx->h_pin);
    if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
    if (ctx->ev_join) (void)hipEventDestroy(ctx->ev_join);
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;  // device buffers are freed by their destructors, on ctx->device
}

extern "C" int sdfnmpc_ctx_device(const sdfnmpc_ctx* ctx) { return ctx ? ctx->device : -1; }

extern "C" int sdfnmpc_dev_alloc(sdfnmpc_ctx* ctx, size_t bytes, void** out) {
    if (!ctx || !out) return fail(SDFNMPC_E_ARG, "NULL argument to sdfnmpc_dev_alloc");
    ScopedDevice sd(ctx->device);
    *out = nullptr;
    HIPCHK(hipMalloc(out, bytes ? bytes : 16));
    return SDFNMPC_OK;
}

extern "C" void sdfnmpc_dev_free(sdfnmpc_ctx* ctx, void* ptr) {
    if (!ctx || !ptr) return;
    ScopedDevice sd(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(ptr);
}

extern "C" int sdfnmpc_memcpy(sdfnmpc_ctx* ctx, void* dst, const void* src, size_t bytes, int kind) {
    if (!ctx || (bytes && (!dst || !src)) || kind < 1 || kind > 3) return fail(SDFNMPC_E_ARG, "bad sdfnmpc_memcpy arguments");
    if (!bytes) return SDFNMPC_OK;
    ScopedDevice sd(ctx->device);
    const hipMemcpyKind k = kind == 1 ? hipMemcpyHostToDevice : kind == 2 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
    HIPCHK(hipMemcpyAsync(dst, src, bytes, k, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return SDFNMPC_OK;
}

// The legacy default (null) stream: PyTorch's default stream has the handle 0, which
// sdfnmpc_ctx_create / _set_stream read as "create a private stream"; this call makes the context
// launch on the null stream itself, so its kernels are ordered with the framework's default-stream work.
extern "C" int sdfnmpc_ctx_use_null_stream(sdfnmpc_ctx* ctx) {
    if (!ctx) return fail(SDFNMPC_E_ARG, "ctx is NULL");
    ScopedDevice sd(ctx->device);
    if (ctx->own_stream) {
        HIPCHK(hipStreamSynchronize(ctx->stream));
        (void)hipStreamDestroy(ctx->stream);
        ctx->own_stream = false;
    }
    ctx->stream = nullptr;
    return SDFNMPC_OK;
}

extern "C" int sdfnmpc_ctx_set_stream(sdfnmpc_ctx* ctx, void* stream) {
    if (!ctx) return fail(SDFNMPC_E_ARG, "ctx is NULL");
    ScopedDevice sd(ctx->device);
    if (ctx->own_stream) {
        HIPCHK(hipStreamSynchronize(ctx->stream));
        (void)hipStreamDestroy(ctx->stream);
        ctx->own_stream = false;
    }
    if (stream) {
        ctx->stream = (hipStream_t)stream;
    } else {
        HIPCHK(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
        ctx->own_stream = true;
    }
    return SDFNMPC_OK;
}

extern "C" void* sdfnmpc_ctx_stream(sdfnmpc_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

extern "C" int sdfnmpc_ctx_synchronize(sdfnmpc_ctx* ctx) {
    if (!ctx) return fail(SDFNMPC_E_ARG, "ctx is NULL");
    ScopedDevice sd(ctx->device);
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return SDFNMPC_OK;
}

extern "C" int sdfnmpc_ctx_set_qp_kernel(sdfnmpc_ctx* ctx, int kernel) {
    if (!ctx) return fail(SDFNMPC_E_ARG, "NULL context");
    if (kernel != SDFNMPC_QP_AUTO && kernel != SDFNMPC_QP_SERIAL && kernel != SDFNMPC_QP_SEGMENTED)
        return fail(SDFNMPC_E_ARG, "qp kernel: SDFNMPC_QP_AUTO, _SERIAL or _SEGMENTED");
    ctx->qp_kernel = kernel;
    return SDFNMPC_OK;
}

static int qp_cset_check(const sdfnmpc_qp_opts* o);
static QpRows qp_rows_of(const sdfnmpc_qp_opts* o);

// AUTO: the segmented kernel for latency-sized batches of long horizons (B <= SDFNMPC_QP_SEG_AUTO_MAX_B,
// N >= SDFNMPC_QP_SEG_AUTO_MIN_N; one workgroup of four wavefronts per instance: 8-10 % lower latency than
// the serial kernel at N = 40, 24 % at N = 60, equal at N = 30, 30 % slower at N = 20 where the three
// couplings outweigh five-node segments), the serial one otherwise (one wavefront per instance: at
// B = 1024 it fills every SIMD once and is 1.6x faster than four wavefronts per instance)
// the segmented kernel covers every row set the serial one does (qp_is_seg_set: 0..3 stage rows, soft or
// hard, and up to QP_NHN terminal rows); the choice between them is the batch / horizon policy below
static int qp_kernel_for(const sdfnmpc_ctx* ctx, int N, int B, bool seg_set) {
    if (!seg_set) return (ctx && N >= 1 && B >= 0) ? SDFNMPC_QP_SERIAL : -1;
    return sdfnmpc_ctx_qp_kernel(ctx, N, B);
}
// a row set the segmented kernel serves (rti_qp_seg.hip: the stage groups of a node on three lanes, the
// nhN terminal rows on lanes 48 + j of the last wave).  T: sdfnmpc_qp_opts or QpArgs (same field names)
template <class T>
static bool qp_is_seg_set(const T& o) {
    return o.nh >= 0 && o.nh <= 3 && o.nhs >= 0 && o.nhs <= o.nh && o.nsN >= 0 && o.nsN <= 3 && o.nhN >= o.nsN &&
           o.nhN <= QP_NHN;
}

extern "C" int sdfnmpc_ctx_qp_kernel(const sdfnmpc_ctx* ctx, int N, int B) {
    if (!ctx || N < 1 || B < 0) return -1;
    if (ctx->qp_kernel == SDFNMPC_QP_SERIAL || !rti_qp_seg_supported(N)) return SDFNMPC_QP_SERIAL;
    if (ctx->qp_kernel == SDFNMPC_QP_SEGMENTED) return SDFNMPC_QP_SEGMENTED;
    // the batch bound doubles from N = 48: the serial kernel then holds two instances per CU instead of
    // four (its LDS), and the segmented one still runs two per CU (measured at N = 60: 2.10 vs 2.67 ms at
    // B = 512; at N = 40, 1.13 vs 1.08 ms at B = 512)
    const int max_b = N >= 48 ? 2 * SDFNMPC_QP_SEG_AUTO_MAX_B : SDFNMPC_QP_SEG_AUTO_MAX_B;
    return (B <= max_b && N >= SDFNMPC_QP_SEG_AUTO_MIN_N) ? SDFNMPC_QP_SEGMENTED : SDFNMPC_QP_SERIAL;
}

extern "C" int sdfnmpc_ctx_qp_kernel_for(const sdfnmpc_ctx* ctx, int N, int B, const sdfnmpc_qp_opts* o) {
    if (o && qp_cset_check(o)) return -1;
    return qp_kernel_for(ctx, N, B, o ? qp_is_seg_set(*o) : true);
}

extern "C" long long sdfnmpc_qp_lds_bytes(int N) {
    return N < 1 ? -1 : (long long)qp_lds_bytes(N);
}

// Instances the context's device solves in one wave of QP workgroups: every CU holds as many
// instances as its LDS fits (the QP keeps each instance's iterate, duals and record window in LDS;
// rti_qp.hip: one 64-lane workgroup per instance, rti_qp_seg.hip: one workgroup of NSEG waves).

extern "C" long long sdfnmpc_qp_capacity(const sdfnmpc_ctx* ctx, int N) { return sdfnmpc_qp_capacity_for(ctx, N, nullptr); }

extern "C" long long sdfnmpc_qp_capacity_for(const sdfnmpc_ctx* ctx, int N, const sdfnmpc_qp_opts* o) {
    if (!ctx || N < 1) return -1;
    if (ctx->n_cu <= 0 || ctx->lds_per_cu == 0) return -1;
    if (o && qp_cset_check(o)) return -1;
    const QpRows rows = o ? qp_rows_of(o) : qp_rows_default();
    // a batch that fills the device: the kernel AUTO picks above SDFNMPC_QP_SEG_AUTO_MAX_B
    const bool seg = qp_kernel_for(ctx, N, 1 << 30, o ? qp_is_seg_set(*o) : true) == SDFNMPC_QP_SEGMENTED;
    const size_t per = seg ? qp_seg_lds_bytes(N) : qp_lds_bytes(N, rows);
    if (per == 0 || per > ctx->lds_per_cu) return 0;  // the horizon does not fit one CU's LDS
    // the runtime's occupancy of the kernel (LDS, registers and waves at once): the serial kernel's 375
    // registers allow one wave per SIMD, four instances per CU, whatever the LDS would admit; the segmented
    // kernel's __launch_bounds__ two or three workgroups per CU
    ScopedDevice sd(ctx->device);
    const int occ = seg ? rti_qp_seg_blocks_per_cu(N) : rti_qp_blocks_per_cu(N, rows);
    const long long by_lds = (long long)(ctx->lds_per_cu / per);
    return (long long)ctx->n_cu * std::min<long long>(by_lds, occ > 0 ? occ : 0);
}

extern "C" int sdfnmpc_ctx_set_tile_rows(sdfnmpc_ctx* ctx, int rows) {
    if (!ctx) return fail(SDFNMPC_E_ARG, "ctx is NULL");
    if (rows != 32 && rows != 64) return fail(SDFNMPC_E_ARG, "tile rows must be 32 or 64");
    ctx->tile_rows = rows;
    return SDFNMPC_OK;
}

extern "C" int sdfnmpc_ctx_enable_timing(sdfnmpc_ctx* ctx, int on) {
    if (!ctx) return fail(SDFNMPC_E_ARG, "ctx is NULL");
    ctx->timing = on != 0;
    return SDFNMPC_OK;
}

static int resolve_stats(sdfnmpc_ctx* ctx) {
    ScopedDevice sd(ctx->device);
    HIPCHK(hipStreamSynchronize(ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->aux));
    for (auto& kv : ctx->stats) {
        for (auto& ev : kv.second.pending) {
            float ms = 0.0f;
            HIPCHK(hipEventElapsedTime(&ms, ev.first, ev.second));
            kv.second.ms += ms;
            kv.second.n += 1;
            (void)hipEventDestroy(ev.first);
            (void)hipEventDestroy(ev.second);
        }
        kv.second.pending.clear();
    }
    return SDFNMPC_OK;
}

extern "C" int sdfnmpc_ctx_kernel_stats(sdfnmpc_ctx* ctx, const char* kernel, double* total_ms, long long* launches) {
    if (!ctx || !kernel) return fail(SDFNMPC_E_ARG, "ctx/kernel is NULL");
    int rc = resolve_stats(ctx);
    if (rc) return rc;
    auto it = ctx->stats.find(kernel);
    if (total_ms) *total_ms = it == ctx->stats.end() ? 0.0 : it->second.ms;
    if (launches) *launches = it == ctx->stats.end() ? 0 : it->second.n;
    return SDFNMPC_OK;
}

extern "C" int sdfnmpc_ctx_reset_stats(sdfnmpc_ctx* ctx) {
    if (!ctx) return fail(SDFNMPC_E_ARG, "ctx is NULL");
    int rc = resolve_stats(ctx);
    if (rc) return rc;
    ctx->stats.clear();
    return SDFNMPC_OK;
}

// ------------------------------------------------------------------------------------------------
// network: .sdfw parsing (sdf-nmpc_amd/weights.py:pack) and packing into the kernels' layouts
namespace {

struct HostNet {
    int nb_states = 3, L = 0, n1 = 0, n2 = 0, n3 = 0, n4 = 0, nf = 0, nd = 0;
    int res = 0;  // 0 'full' [h2 | e | z], 1 'state' [h2 | e], 2 'latent' [h2 | z], 3 plain MLP [h2] into layer 3
                  // (neural_df.py:76-78: any other `res` value)
    int act = 0;  // 0 sin(w0 .), 1 relu, 2 softplus (neural_df.py:40-47)
    float w0 = 0, max_df = 1;
    std::vector<float> dirs, freqs;                           // [3][nd], [nf]
    std::vector<float> W1, b1, W2, b2, W3, b3, W4, b4, W5, b5;  // torch order / shapes
    int E() const { return 3 + 2 * nd * nf; }
    bool e3() const { return res == 0 || res == 1; }  // layer 3 sees the embedding
    bool z3() const { return res == 0 || res == 2; }  // layer 3 sees the latent
    int c3() const { return n2 + (e3() ? E() : 0) + (z3() ? L : 0); }  // W3 row length
};

uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
// identical to weights.prng_uniform / oracle orc_prng_uniform
void prng_fill(uint64_t seed, uint64_t stream, std::vector<double>& out) {
    const uint64_t key = mix64(seed * 0x9E3779B97F4A7C15ULL + stream * 0xD1B54A32D192ED03ULL + 1ULL);
    for (size_t i = 0; i < out.size(); ++i)
        out[i] = (double)(mix64(key + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ULL) >> 40) * (1.0 / 16777216.0);
}

std::vector<float*> param_list(HostNet& h) {
    return {h.W1.data(), h.b1.data(), h.W2.data(), h.b2.data(), h.W3.data(),
            h.b3.data(), h.W4.data(), h.b4.data(), h.W5.data(), h.b5.data()};
}
std::vector<std::pair<int, int>> param_shapes(const HostNet& h) {
    const int E = h.E(), L = h.L;
    return {{h.n1, E + L}, {h.n1, 1}, {h.n2, h.n1}, {h.n2, 1}, {h.n3, h.c3()},
            {h.n3, 1},     {h.n4, h.n3}, {h.n4, 1}, {1, h.n4}, {1, 1}};
}
void alloc_params(HostNet& h) {
    auto sh = param_shapes(h);
    std::vector<std::vector<float>*> v = {&h.W1, &h.b1, &h.W2, &h.b2, &h.W3, &h.b3, &h.W4, &h.b4, &h.W5, &h.b5};
    for (size_t i = 0; i < v.size(); ++i) v[i]->assign((size_t)sh[i].first * sh[i].second, 0.0f);
}

// The deployed NeuralDF (layers [256,256,128,64], 'oct' x 5 frequencies, res 'full', sin) runs the fused
// sdf_mlp.hip / sdf_row.hip kernels.  Every other architecture -- config C5's [1024,1024,512,256], and the
// reference's variants: any layer sizes (zero-padded to multiples of 128: the padded units' outgoing
// weights are zero, so they change nothing), embeddings none / pos / cube / oct / dod / ico with any
// frequency count, res full / state / latent / none (a plain MLP), any size_latent, activations sin / relu /
// softplus -- runs the layer-by-layer
// GEMM schedule of sdf_wide.hip ("wide" below means exactly that: not the deployed net).
bool is_deployed(const HostNet& h) {
    return h.n1 == N1 && h.n2 == N2 && h.n3 == N3 && h.n4 == N4 && h.nd == EMB_ND && h.nf == EMB_NF && h.res == 0 &&
           h.act == 0 && h.L == L;
}
bool is_wide(const HostNet& h) { return !is_deployed(h); }
int pad128(int n) { return (n + 127) / 128 * 128; }

constexpr int L_MAX = 1024;  // size_latent bound (the wide schedule pads it to a multiple of 128)
int check_supported(const HostNet& h) {
    if (h.nb_states != 3 || h.L < 1 || h.L > L_MAX || h.E() > 256 || h.res < 0 || h.res > 3 || h.act < 0 || h.act > 2) {
        char buf[256];
        snprintf(buf, sizeof buf,
                 "network architecture (states %d, latent %d, embedding features %d, res %d, act %d) is not built "
                 "for; this build supports 3 states, latent 1..%d, at most 256 embedding features",
                 h.nb_states, h.L, h.E(), h.res, h.act, L_MAX);
        return fail(SDFNMPC_E_UNSUPPORTED, buf);
    }
    return SDFNMPC_OK;
}

int parse_sdfw(const void* blob, size_t bytes, HostNet& h) {
    // version 1: magic, version, nb_states, L, n1..n4, nb_freqs, n_dirs, res (0), w0, max_df;
    // version 2 adds the activation after res (sdf_nmpc_amd/weights.py)
    const unsigned char* p = (const unsigned char*)blob;
    if (!blob || bytes < 12 || memcmp(p, "SDFNMPCW", 8) != 0) return fail(SDFNMPC_E_FORMAT, "not an .sdfw blob");
    uint32_t ver = 0;
    memcpy(&ver, p + 8, 4);
    if (ver != 1 && ver != 2) return fail(SDFNMPC_E_FORMAT, "unsupported .sdfw version");
    const int nu = ver == 1 ? 10 : 11;
    const size_t HDR = 8 + nu * 4 + 2 * 4;
    if (bytes < HDR) return fail(SDFNMPC_E_FORMAT, "truncated .sdfw header");
    uint32_t u[11] = {};
    memcpy(u, p + 8, (size_t)nu * 4);
    float f[2];
    memcpy(f, p + 8 + nu * 4, sizeof f);
    if (ver == 1 && u[9] != 0) return fail(SDFNMPC_E_FORMAT, "version-1 .sdfw blobs are res='full'");
    h.res = (int)u[9];
    h.act = ver == 2 ? (int)u[10] : 0;
    h.nb_states = (int)u[1];
    h.L = (int)u[2];
    h.n1 = (int)u[3]; h.n2 = (int)u[4]; h.n3 = (int)u[5]; h.n4 = (int)u[6];
    h.nf = (int)u[7];
    h.nd = (int)u[8];
    h.w0 = f[0];
    h.max_df = f[1];
    if (h.nd < 0 || h.nf < 0 || h.nd > 64 || h.nf > 64 || (h.nd == 0) != (h.nf == 0) || h.L < 0 || h.n1 <= 0 ||
        h.n2 <= 0 || h.n3 <= 0 || h.n4 <= 0 || h.n1 > 65536 || h.n2 > 65536 || h.n3 > 65536 || h.n4 > 65536)
        return fail(SDFNMPC_E_FORMAT, "bad .sdfw header");
    size_t off = HDR;
    auto take = [&](std::vector<float>& v, size_t n) -> bool {
        if (off + 4 * n > bytes) return false;
        v.resize(n);
        memcpy(v.data(), p + off, 4 * n);
        off += 4 * n;
        return true;
    };
    if (!take(h.dirs, (size_t)3 * h.nd) || !take(h.freqs, (size_t)h.nf)) return fail(SDFNMPC_E_FORMAT, "truncated");
    auto sh = param_shapes(h);
    std::vector<std::vector<float>*> v = {&h.W1, &h.b1, &h.W2, &h.b2, &h.W3, &h.b3, &h.W4, &h.b4, &h.W5, &h.b5};
    for (size_t i = 0; i < v.size(); ++i)
        if (!take(*v[i], (size_t)sh[i].first * sh[i].second)) return fail(SDFNMPC_E_FORMAT, "truncated .sdfw params");
    if (off != bytes) return fail(SDFNMPC_E_FORMAT, "trailing bytes in .sdfw blob");
    return check_supported(h);
}

void siren_host(HostNet& h, uint64_t seed, float wg, float bg) {
    h.nb_states = 3; h.L = L; h.n1 = N1; h.n2 = N2; h.n3 = N3; h.n4 = N4; h.nf = EMB_NF; h.nd = EMB_ND;
    h.w0 = 20.0f;
    h.max_df = 1.0f;
    // 'oct' dirs exactly as torch builds them (embeddings.py:37-51): +-1 / fp32 sqrt(3)
    static const int sg[8][3] = {{-1, -1, -1}, {-1, -1, 1}, {-1, 1, -1}, {-1, 1, 1},
                                 {1, -1, -1},  {1, -1, 1},  {1, 1, -1},  {1, 1, 1}};
    const float nrm = sqrtf(3.0f);
    h.dirs.assign(3 * 8, 0.0f);
    for (int d = 0; d < 8; ++d)
        for (int c = 0; c < 3; ++c) h.dirs[c * 8 + d] = (float)sg[d][c] / nrm;
    h.freqs = {1.0f, 2.0f, 4.0f, 8.0f, 16.0f};
    alloc_params(h);
    auto ptr = param_list(h);
    auto sh = param_shapes(h);
    std::vector<double> u;
    for (int t = 0; t < 10; t += 2) {
        const double bound = std::sqrt(6.0 / sh[t].second) / (double)h.w0;
        u.assign((size_t)sh[t].first * sh[t].second, 0.0);
        prng_fill(seed, t, u);
        for (size_t i = 0; i < u.size(); ++i) ptr[t][i] = (float)((2.0 * u[i] - 1.0) * (bound * (double)wg));
        if (bg > 0.0f) {
            u.assign((size_t)sh[t + 1].first * sh[t + 1].second, 0.0);
            prng_fill(seed, t + 1, u);
            for (size_t i = 0; i < u.size(); ++i) ptr[t + 1][i] = (float)((2.0 * u[i] - 1.0) * (bound * (double)bg));
        }
    }
}

template <typename F>
void pack_operand(std::vector<float>& dst, int N, int K, F&& W) {
    const int CB = (N + 31) / 32, G = K / 8;
    const size_t base = dst.size();
    dst.resize(base + packed_floats(N, K), 0.0f);
    for (int cb = 0; cb < CB; ++cb)
        for (int g = 0; g < G; ++g)
            for (int ln = 0; ln < 64; ++ln)
                for (int i = 0; i < 4; ++i) {
                    const int j = cb * 32 + (ln & 31), k = (ln >> 5) * (K / 2) + 4 * g + i;
                    dst[base + (((size_t)cb * G + g) * 64 + ln) * 4 + i] = (j < N) ? W(j, k) : 0.0f;
                }
}

}  // namespace

struct WideDev {  // plain row-major [N][K] fp32 operands of the wide schedule (sdf_wide.hip)
    const float *F1 = nullptr, *F2 = nullptr, *F3 = nullptr, *F4 = nullptr;
    const float *B4 = nullptr, *B3h = nullptr, *B3e = nullptr, *B2 = nullptr, *B1e = nullptr;
    const float *Bz = nullptr, *Hz = nullptr, *bz = nullptr, *b2 = nullptr, *b4 = nullptr, *w5 = nullptr;
    const float4* emb_tab = nullptr;
    int P1 = 0, P2 = 0, P3 = 0, P4 = 0;  // layer widths padded to multiples of 128
    int NEK = NE, NEB = 128;             // embedding width as a K segment / as the d e GEMMs' output
    int nb = 0;                          // projected frequencies (n_dirs x nb_freqs)
    int LH = L, LZ = L;                  // size_latent, and padded to a multiple of 128 (the GEMMs' K / N)
    bool e3 = true;                      // layer 3 sees the embedding (res 'full' / 'state')
    int act = 0;                         // 0 sin, 1 relu, 2 softplus
};

struct sdfnmpc_net {
    int device = 0;
    HostNet host;
    void* dmem = nullptr;
    SdfArgs args{};  // weight pointers filled; per-call fields left zero
    SdfRowArgs row{};  // the single-row path's weight pointers (deployed architecture only)
    const float4* WzT = nullptr;
    const float* bias13 = nullptr;
    uint64_t fingerprint = 0;
    bool wide = false;
    WideDev wd;
    WideRowArgs wrow{};    // the row evaluator's operands (sdf_row_wide.hip); per-call fields left zero
    bool wrow_ok = false;  // the row evaluator and its server fit this network (LDS, weight bytes)
    // process-unique id: caches keyed on a network (the host path's hoist) never confuse a freed
    // network with a new one allocated at the same address
    uint64_t uid = next_uid();
    static uint64_t next_uid() {
        static std::atomic<uint64_t> n{1};
        return n++;
    }
};

// [width] float4 (dir * 2^f, 0) of embedding feature m: the projected frequencies in the reference's order
// (embeddings.py:108-109: direction-major, frequency-minor; the sin half, then the same for the shifted half)
static void emb_table(const HostNet& h, std::vector<float>& blob, int width = NE) {
    const int nb = h.nd * h.nf, E = h.E();
    for (int m = 0; m < width; ++m) {
        float v[4] = {0, 0, 0, 0};
        int j = -1;
        if (m >= 3 && m < 3 + nb) j = m - 3;
        else if (m >= 3 + nb && m < E) j = m - 3 - nb;
        if (j >= 0) {
            const int d = j / h.nf, f = j % h.nf;
            for (int c = 0; c < 3; ++c) v[c] = h.dirs[c * h.nd + d] * h.freqs[f];  // freq = 2^f: exact
        }
        blob.insert(blob.end(), v, v + 4);
    }
}

static uint64_t net_fingerprint(HostNet& h) {  // FNV-1a over the parameters in torch order
    uint64_t fp = 1469598103934665603ULL;
    auto sh = param_shapes(h);
    auto pl = param_list(h);
    for (size_t t = 0; t < pl.size(); ++t) {
        const unsigned char* b = (const unsigned char*)pl[t];
        const size_t nb = (size_t)sh[t].first * sh[t].second * 4;
        for (size_t q = 0; q < nb; ++q) fp = (fp ^ b[q]) * 1099511628211ULL;
    }
    return fp;
}

// weight bytes up to which a variant network takes the row evaluator on the host path
// (SDFNMPC_WIDE_ROW_MAX_MB overrides; 0 sends every variant to the layer-by-layer schedule)
static size_t wide_row_weight_cap() {
    if (const char* e = getenv("SDFNMPC_WIDE_ROW_MAX_MB")) return (size_t)(atof(e) * 1048576.0);
    return (size_t)64 << 20;
}

static int upload_wide(sdfnmpc_ctx* ctx, HostNet&& h, sdfnmpc_net** out) {
    // layer widths zero-padded to multiples of 128 (the GEMM's column tile), the embedding to NEK (a
    // multiple of 32) as a K segment and to NEB (a multiple of 128) as the d e GEMMs' output width
    const int n1 = h.n1, n2 = h.n2, n3 = h.n3, n4 = h.n4, E = h.E(), Lh = h.L, LZ = pad128(Lh), c1 = E + Lh, c3 = h.c3();
    const int P1 = pad128(n1), P2 = pad128(n2), P3 = pad128(n3), P4 = pad128(n4);
    const int NEK = std::max(96, (E + 31) / 32 * 32), NEB = pad128(E);
    const bool e3 = h.e3(), z3 = h.z3();
    const int z3off = n2 + (e3 ? E : 0);  // first latent column of W3
    const float *W1 = h.W1.data(), *W2 = h.W2.data(), *W3 = h.W3.data(), *W4 = h.W4.data();
    std::vector<float> blob;
    std::vector<size_t> off;
    auto mat = [&](int N, int K, auto&& f) {
        off.push_back(blob.size());
        for (int j = 0; j < N; ++j)
            for (int k = 0; k < K; ++k) blob.push_back(f(j, k));
    };
    auto vec = [&](const std::vector<float>& v, int P) {
        off.push_back(blob.size());
        blob.insert(blob.end(), v.begin(), v.end());
        blob.insert(blob.end(), (size_t)(P - (int)v.size()), 0.0f);
    };
    mat(P1, NEK, [&](int j, int k) { return j < n1 && k < E ? W1[(size_t)j * c1 + k] : 0.0f; });                // F1
    mat(P2, P1, [&](int j, int k) { return j < n2 && k < n1 ? W2[(size_t)j * n1 + k] : 0.0f; });                 // F2
    mat(P3, P2 + (e3 ? NEK : 0), [&](int j, int k) {                                                             // F3
        if (j >= n3) return 0.0f;
        if (k < P2) return k < n2 ? W3[(size_t)j * c3 + k] : 0.0f;
        return k - P2 < E ? W3[(size_t)j * c3 + n2 + (k - P2)] : 0.0f;
    });
    mat(P4, P3, [&](int j, int k) { return j < n4 && k < n3 ? W4[(size_t)j * n3 + k] : 0.0f; });                 // F4
    mat(P3, P4, [&](int j, int k) { return j < n3 && k < n4 ? W4[(size_t)k * n3 + j] : 0.0f; });                 // B4
    mat(P2, P3, [&](int j, int k) { return j < n2 && k < n3 ? W3[(size_t)k * c3 + j] : 0.0f; });                 // B3h
    mat(NEB, P3, [&](int j, int k) { return e3 && j < E && k < n3 ? W3[(size_t)k * c3 + n2 + j] : 0.0f; });      // B3e
    mat(P1, P2, [&](int j, int k) { return j < n1 && k < n2 ? W2[(size_t)k * n1 + j] : 0.0f; });                 // B2
    mat(NEB, P1, [&](int j, int k) { return j < E && k < n1 ? W1[(size_t)k * c1 + j] : 0.0f; });                 // B1e
    mat(LZ, P1 + P3, [&](int j, int k) {  // Bz: d z = [delta1 | delta3] . [W1z ; W3z] (the 131-wide jac_sdf_l4c)
        if (j >= Lh) return 0.0f;
        if (k < P1) return k < n1 ? W1[(size_t)k * c1 + E + j] : 0.0f;
        return z3 && k - P1 < n3 ? W3[(size_t)(k - P1) * c3 + z3off + j] : 0.0f;
    });
    mat(P1 + P3, LZ, [&](int j, int k) {                                                                         // Hz
        if (k >= Lh) return 0.0f;
        if (j < P1) return j < n1 ? W1[(size_t)j * c1 + E + k] : 0.0f;
        return z3 && j - P1 < n3 ? W3[(size_t)(j - P1) * c3 + z3off + k] : 0.0f;
    });
    off.push_back(blob.size());  // bz = [b1 | b3], padded
    blob.insert(blob.end(), h.b1.begin(), h.b1.end());
    blob.insert(blob.end(), (size_t)(P1 - n1), 0.0f);
    blob.insert(blob.end(), h.b3.begin(), h.b3.end());
    blob.insert(blob.end(), (size_t)(P3 - n3), 0.0f);
    vec(h.b2, P2);
    vec(h.b4, P4);
    vec(h.W5, P4);
    while (blob.size() % 4) blob.push_back(0.0f);
    off.push_back(blob.size());
    emb_table(h, blob, NEK);
    for (size_t o : off)
        if (o % 4) return fail(SDFNMPC_E_FORMAT, "internal: misaligned wide operand");
    auto* net = new sdfnmpc_net();
    net->device = ctx->device;
    net->wide = true;
    ScopedDevice sd(ctx->device);
    if (hipMalloc(&net->dmem, blob.size() * sizeof(float)) != hipSuccess ||
        hipMemcpy(net->dmem, blob.data(), blob.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) {
        if (net->dmem) (void)hipFree(net->dmem);
        delete net;
        return fail(SDFNMPC_E_HIP, "wide net: device upload failed");
    }
    const float* d = (const float*)net->dmem;
    WideDev& w = net->wd;
    int i = 0;
    w.F1 = d + off[i++]; w.F2 = d + off[i++]; w.F3 = d + off[i++]; w.F4 = d + off[i++];
    w.B4 = d + off[i++]; w.B3h = d + off[i++]; w.B3e = d + off[i++]; w.B2 = d + off[i++]; w.B1e = d + off[i++];
    w.Bz = d + off[i++];
    w.Hz = d + off[i++]; w.bz = d + off[i++]; w.b2 = d + off[i++]; w.b4 = d + off[i++]; w.w5 = d + off[i++];
    w.emb_tab = (const float4*)(d + off[i++]);
    w.P1 = P1; w.P2 = P2; w.P3 = P3; w.P4 = P4; w.NEK = NEK; w.NEB = NEB;
    w.nb = h.nd * h.nf; w.e3 = e3; w.act = h.act; w.LH = Lh; w.LZ = LZ;
    net->args.b5 = h.b5[0];
    net->args.w0 = h.w0;
    WideRowArgs& ra = net->wrow;
    ra.F1 = w.F1; ra.F2 = w.F2; ra.F3 = w.F3; ra.F4 = w.F4;
    ra.B4 = w.B4; ra.B3h = w.B3h; ra.B3e = w.B3e; ra.B2 = w.B2; ra.B1e = w.B1e;
    ra.Bz = w.Bz; ra.Hz = w.Hz; ra.bz = w.bz; ra.b2 = w.b2; ra.b4 = w.b4; ra.w5 = w.w5; ra.emb_tab = w.emb_tab;
    ra.b5 = h.b5[0]; ra.w0 = h.w0;
    ra.P1 = P1; ra.P2 = P2; ra.P3 = P3; ra.P4 = P4; ra.NEK = NEK; ra.NEB = NEB; ra.nb = w.nb;
    ra.LH = Lh; ra.LZ = LZ; ra.e3 = e3 ? 1 : 0; ra.act = h.act;
    // one workgroup per row streams every weight once per row: worth it while the weights are L2 / MALL
    // sized (a C5-sized network is faster on the layer-by-layer GEMMs)
    const size_t srv_lds = wide_row_lds_bytes(ra) + 2 * SDF_MBOX_FLOATS * sizeof(float);
    net->wrow_ok = srv_lds <= 160 * 1024 && blob.size() * sizeof(float) <= wide_row_weight_cap();
    net->fingerprint = net_fingerprint(h);
    net->host = std::move(h);
    *out = net;
    return SDFNMPC_OK;
}

static int upload_net(sdfnmpc_ctx* ctx, HostNet&& h, sdfnmpc_net** out) {
    if (is_wide(h)) return upload_wide(ctx, std::move(h), out);
    const int Ein = h.E(), Lh = h.L;
    const float* W1 = h.W1.data();
    const float* W2 = h.W2.data();
    const float* W3 = h.W3.data();
    const float* W4 = h.W4.data();
    const int c1 = Ein + Lh, c3 = N2 + Ein + Lh;  // row lengths of W1, W3
    std::vector<float> blob;
    std::vector<size_t> off;
    auto mark = [&]() { off.push_back(blob.size()); };
    mark(); pack_operand(blob, N1, KE, [&](int j, int k) { return k < E ? W1[(size_t)j * c1 + k] : 0.0f; });
    mark(); pack_operand(blob, N2, N1, [&](int j, int k) { return W2[(size_t)j * N1 + k]; });
    mark(); pack_operand(blob, N3, N2, [&](int j, int k) { return W3[(size_t)j * c3 + k]; });
    mark(); pack_operand(blob, N3, KE, [&](int j, int k) { return k < E ? W3[(size_t)j * c3 + N2 + k] : 0.0f; });
    mark(); pack_operand(blob, N4, N3, [&](int j, int k) { return W4[(size_t)j * N3 + k]; });
    mark(); pack_operand(blob, N3, N4, [&](int j, int k) { return W4[(size_t)k * N3 + j]; });
    mark(); pack_operand(blob, N2, N3, [&](int j, int k) { return W3[(size_t)k * c3 + j]; });
    mark(); pack_operand(blob, NE, N3, [&](int j, int k) { return j < E ? W3[(size_t)k * c3 + N2 + j] : 0.0f; });
    mark(); pack_operand(blob, N1, N2, [&](int j, int k) { return W2[(size_t)k * N1 + j]; });
    mark(); pack_operand(blob, NE, N1, [&](int j, int k) { return j < E ? W1[(size_t)k * c1 + j] : 0.0f; });
    mark(); pack_operand(blob, L, N3, [&](int j, int k) { return W3[(size_t)k * c3 + N2 + E + j]; });
    mark(); pack_operand(blob, L, N1, [&](int j, int k) { return W1[(size_t)k * c1 + E + j]; });
    // hoist operand Wsrc(j, k) = [W1[:, E:] ; W3[:, N2+E:]](j, k): N = C13_STRIDE, K = L
    mark();
    pack_operand(blob, C13_STRIDE, L, [&](int j, int k) {
        return j < N1 ? W1[(size_t)j * c1 + E + k] : W3[(size_t)(j - N1) * c3 + N2 + E + k];
    });
    mark(); for (int j = 0; j < N1; ++j) blob.push_back(h.b1[j]); for (int j = 0; j < N3; ++j) blob.push_back(h.b3[j]);
    mark(); blob.insert(blob.end(), h.b2.begin(), h.b2.end());
    mark(); blob.insert(blob.end(), h.b4.begin(), h.b4.end());
    mark(); blob.insert(blob.end(), h.W5.begin(), h.W5.end());
    while (blob.size() % 4) blob.push_back(0.0f);
    mark();
    emb_table(h, blob);
    // plain torch-layout copies for the single-row latency path (sdf_row.hip)
    auto plain = [&](const std::vector<float>& v) {
        mark();
        blob.insert(blob.end(), v.begin(), v.end());
        while (blob.size() % 4) blob.push_back(0.0f);
    };
    auto padded = [&](const std::vector<float>& v, int J, int K) {  // rows padded to a multiple of 4 floats
        const int K4 = (K + 3) / 4 * 4;
        std::vector<float> t((size_t)J * K4, 0.0f);
        for (int j = 0; j < J; ++j)
            for (int k = 0; k < K; ++k) t[(size_t)j * K4 + k] = v[(size_t)j * K + k];
        plain(t);
    };
    padded(h.W1, N1, c1); padded(h.W2, N2, N1); padded(h.W3, N3, c3); padded(h.W4, N4, N3);
    auto transposed = [&](const std::vector<float>& v, int J, int K) {
        std::vector<float> t((size_t)J * K);
        for (int j = 0; j < J; ++j)
            for (int k = 0; k < K; ++k) t[(size_t)k * J + j] = v[(size_t)j * K + k];
        plain(t);
    };
    transposed(h.W1, N1, c1); transposed(h.W2, N2, N1); transposed(h.W3, N3, c3); transposed(h.W4, N4, N3);
    for (size_t o : off)
        if (o % 4) return fail(SDFNMPC_E_FORMAT, "internal: misaligned packed operand");

    auto* net = new sdfnmpc_net();
    net->device = ctx->device;
    ScopedDevice sd(ctx->device);
    hipError_t e = hipMalloc(&net->dmem, blob.size() * sizeof(float));
    if (e != hipSuccess) {
        delete net;
        return fail(SDFNMPC_E_HIP, std::string("hipMalloc(net): ") + hipGetErrorString(e));
    }
    e = hipMemcpy(net->dmem, blob.data(), blob.size() * sizeof(float), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(net->dmem);
        delete net;
        return fail(SDFNMPC_E_HIP, std::string("hipMemcpy(net): ") + hipGetErrorString(e));
    }
    const float* d = (const float*)net->dmem;
    SdfArgs& a = net->args;
    int i = 0;
    a.wF1 = (const float4*)(d + off[i++]);
    a.wF2 = (const float4*)(d + off[i++]);
    a.wF3h = (const float4*)(d + off[i++]);
    a.wF3e = (const float4*)(d + off[i++]);
    a.wF4 = (const float4*)(d + off[i++]);
    a.wB4 = (const float4*)(d + off[i++]);
    a.wB3 = (const float4*)(d + off[i++]);
    a.wB3e = (const float4*)(d + off[i++]);
    a.wB2 = (const float4*)(d + off[i++]);
    a.wB1e = (const float4*)(d + off[i++]);
    a.wB3z = (const float4*)(d + off[i++]);
    a.wB1z = (const float4*)(d + off[i++]);
    net->WzT = (const float4*)(d + off[i++]);
    net->bias13 = d + off[i++];
    a.b2 = d + off[i++];
    a.b4 = d + off[i++];
    a.w5 = d + off[i++];
    a.emb_tab = (const float4*)(d + off[i++]);
    a.b5 = h.b5[0];
    a.w0 = h.w0;
    SdfRowArgs& ra = net->row;
    ra.W1 = d + off[i++];
    ra.W2 = d + off[i++];
    ra.W3 = d + off[i++];
    ra.W4 = d + off[i++];
    ra.W1T = d + off[i++];
    ra.W2T = d + off[i++];
    ra.W3T = d + off[i++];
    ra.W4T = d + off[i++];
    ra.b1 = net->bias13;
    ra.b3 = net->bias13 + N1;
    ra.b2 = a.b2;
    ra.b4 = a.b4;
    ra.w5 = a.w5;
    ra.b5 = a.b5;
    ra.w0 = a.w0;
    ra.emb_tab = a.emb_tab;
    const uint64_t fp = net_fingerprint(h);
    net->fingerprint = fp;
    net->host = std::move(h);
    *out = net;
    return SDFNMPC_OK;
}

extern "C" int sdfnmpc_net_load(sdfnmpc_ctx* ctx, const void* blob, size_t bytes, sdfnmpc_net** out) {
    if (!ctx || !out) return fail(SDFNMPC_E_ARG, "ctx/out is NULL");
    HostNet h;
    int rc = parse_sdfw(blob, bytes, h);
    if (rc) return rc;
    return upload_net(ctx, std::move(h), out);
}

extern "C" int sdfnmpc_net_load_file(sdfnmpc_ctx* ctx, const char* path, sdfnmpc_net** out) {
    if (!ctx || !path || !out) return fail(SDFNMPC_E_ARG, "NULL argument");
    FILE* f = fopen(path, "rb");
    if (!f) return fail(SDFNMPC_E_ARG, std::string("cannot open ") + path);
    std::vector<unsigned char> buf;
    unsigned char tmp[1 << 16];
    size_t n;
    while ((n = fread(tmp, 1, sizeof tmp, f)) > 0) buf.insert(buf.end(), tmp, tmp + n);
    fclose(f);
    return sdfnmpc_net_load(ctx, buf.data(), buf.size(), out);
}

extern "C" int sdfnmpc_net_siren(sdfnmpc_ctx* ctx, uint64_t seed, float wg, float bg, sdfnmpc_net** out) {
    if (!ctx || !out) return fail(SDFNMPC_E_ARG, "ctx/out is NULL");
    HostNet h;
    siren_host(h, seed, wg, bg);
    return upload_net(ctx, std::move(h), out);
}

// networks an abandoned SDF server (srv_stop timeout) may still be reading: never freed
static std::mutex g_abandoned_mu;
static std::vector<uint64_t> g_abandoned_nets;
static void mark_abandoned(uint64_t uid) {
    std::lock_guard<std::mutex> lk(g_abandoned_mu);
    g_abandoned_nets.push_back(uid);
}

extern "C" void sdfnmpc_net_free(sdfnmpc_net* net) {
    if (!net) return;
    {
        std::lock_guard<std::mutex> lk(g_abandoned_mu);
        // hipFree would also synchronise the device, i.e. wait for the very server that refused to stop
        if (std::find(g_abandoned_nets.begin(), g_abandoned_nets.end(), net->uid) != g_abandoned_nets.end()) return;
    }
    ScopedDevice sd(net->device);
    if (net->dmem) (void)hipFree(net->dmem);
    delete net;
}

extern "C" float sdfnmpc_net_max_df(const sdfnmpc_net* net) { return net ? net->host.max_df : NAN; }
extern "C" int sdfnmpc_net_size_latent(const sdfnmpc_net* net) { return net ? net->host.L : -1; }
extern "C" uint64_t sdfnmpc_net_fingerprint(const sdfnmpc_net* net) { return net ? net->fingerprint : 0; }

// ------------------------------------------------------------------------------------------------
// SDF evaluation
static int run_sdf(sdfnmpc_ctx* ctx, const sdfnmpc_net* net, long long rows, const float4* pos4, const float* c13,
                   int rows_per_inst, float4* out4, float* glat, int M, const SdfArgs* cons = nullptr) {
    if (rows > 0x7fffffffLL / 2) return fail(SDFNMPC_E_ARG, "too many rows");
    SdfArgs a = net->args;
    if (cons) {
        a.x = cons->x;
        a.p = cons->p;
        a.np = cons->np;
        a.h = cons->h;
        a.Jh = cons->Jh;
        a.max_df = cons->max_df;
    }
    a.c13 = c13;
    a.pos = pos4;
    a.out = out4;
    a.grad_latent = glat;
    a.rows = (int)rows;
    a.rows_per_inst = rows_per_inst;
    HIPCHK(timed(ctx, "sdf_mlp", [&] { return launch_sdf_mlp(a, M, glat != nullptr, ctx->stream); }));
    return SDFNMPC_OK;
}

// wide schedule (sdf_wide.hip): hoist, embedding, 4 forward + 5 backward GEMMs, final contraction.
// Latent: fp32 [n_inst][L] (zf) or fp64 at a stride (zd, the stage parameters).  Geometry: pos4, or
// x / p (then also the constraint epilogue when cons->h is set).
static int run_wide(sdfnmpc_ctx* ctx, const sdfnmpc_net* net, long long rows, const float4* pos4, const float* zf,
                    const double* zd, long long zstride, int n_inst, int rows_per_inst, float4* out4,
                    const SdfArgs* cons, float* glat = nullptr) {
    if (rows > 0x7fffffffLL / 2) return fail(SDFNMPC_E_ARG, "too many rows");
    const WideDev& w = net->wd;
    const int n1 = w.P1, n2 = w.P2, n3 = w.P3, n4 = w.P4, nz = n1 + n3, R = (int)rows;
    const int NEK = w.NEK, NEB = w.NEB, LH = w.LH, LZ = w.LZ;
    const bool zpad = LH != LZ;  // size_latent not a multiple of 128: padded latent and d z staging
    const size_t per_row = 2 * (size_t)NEK + 2 * (size_t)(n1 + n2 + n3 + n4) + 2 * (size_t)NEB +
                           (zpad && glat ? (size_t)LZ : 0);
    const size_t nfl = per_row * rows + (size_t)n_inst * (LZ + nz);
    HIPCHK(ctx->wws.ensure(nfl * sizeof(float)));
    float* q = (float*)ctx->wws.p;
    auto take = [&](size_t n) { float* r = q; q += n; return r; };
    float *Eb = take((size_t)R * NEK), *Gb = take((size_t)R * NEK);
    float *H1 = take((size_t)R * n1), *D1 = take((size_t)R * n1), *H2 = take((size_t)R * n2), *D2 = take((size_t)R * n2);
    float *H3 = take((size_t)R * n3), *D3 = take((size_t)R * n3), *H4 = take((size_t)R * n4), *D4 = take((size_t)R * n4);
    float *GE3 = take((size_t)R * NEB), *GE1 = take((size_t)R * NEB);
    float* z = take((size_t)n_inst * LZ);
    float* c13 = take((size_t)n_inst * nz);
    float* gz = (zpad && glat) ? take((size_t)R * LZ) : glat;  // d df / d z before its padding is cut off
    hipStream_t st = ctx->stream;
    if (zd) {
        HIPCHK(timed(ctx, "sdf_wide_hoist", [&] { return launch_wide_latent<double>(zd, zstride, n_inst, LH, LZ, z, st); }));
        zf = z;
    } else if (zpad) {  // fp32 [n_inst][LH] -> [n_inst][LZ]
        HIPCHK(timed(ctx, "sdf_wide_hoist", [&] { return launch_wide_latent<float>(zf, LH, n_inst, LH, LZ, z, st); }));
        zf = z;
    }
    const float w0 = net->args.w0;
    auto gemm = [&](const float* A1, int K1, const float* A2, int K2, const float* W, int M, int N, int epi,
                    const float* bias, const float* c, const float* d, int ldd, float* o1, float* o2,
                    const char* name) -> hipError_t {
        WideGemmArgs g{};
        g.A1 = A1; g.lda1 = K1; g.K1 = K1;
        g.A2 = A2; g.lda2 = K2; g.K2 = K2;
        g.W = W; g.M = M; g.N = N;
        g.bias = bias; g.c = c; g.ldc = nz; g.rows_per_inst = rows_per_inst;
        g.d = d; g.ldd = ldd; g.w5 = w.w5;
        g.out1 = o1; g.ld1 = N; g.out2 = o2; g.ld2 = N; g.w0 = w0; g.act = w.act;
        return timed(ctx, name, [&] { return launch_wide_gemm(g, epi, st); });
    };
    HIPCHK(gemm(zf, LZ, nullptr, 0, w.Hz, n_inst, nz, WIDE_EPI_STORE, w.bz, nullptr, nullptr, 0, c13, nullptr,
                "sdf_wide_hoist"));
    WideSdfArgs ea{};
    ea.rows = R; ea.n4 = n4; ea.pos = pos4; ea.emb_tab = w.emb_tab; ea.E = Eb; ea.G = Gb;
    ea.nb = w.nb; ea.nek = NEK; ea.neb = NEB;
    if (cons) { ea.x = cons->x; ea.p = cons->p; ea.np = cons->np; ea.h = cons->h; ea.Jh = cons->Jh; ea.max_df = cons->max_df; }
    HIPCHK(timed(ctx, "sdf_wide_emb", [&] { return launch_wide_emb(ea, st); }));
    // forward: L1..L4 (layer 3 sees [h2 | e] for res full / state; its latent part is in c13)
    HIPCHK(gemm(Eb, NEK, nullptr, 0, w.F1, R, n1, WIDE_EPI_SIN, nullptr, c13, nullptr, 0, H1, D1, "sdf_wide_gemm"));
    HIPCHK(gemm(H1, n1, nullptr, 0, w.F2, R, n2, WIDE_EPI_SIN, w.b2, nullptr, nullptr, 0, H2, D2, "sdf_wide_gemm"));
    HIPCHK(gemm(H2, n2, w.e3 ? Eb : nullptr, w.e3 ? NEK : 0, w.F3, R, n3, WIDE_EPI_SIN, nullptr, c13 + n1, nullptr, 0,
                H3, D3, "sdf_wide_gemm"));
    HIPCHK(gemm(H3, n3, nullptr, 0, w.F4, R, n4, WIDE_EPI_SIN_L4, w.b4, nullptr, nullptr, 0, H4, D4, "sdf_wide_gemm"));
    // backward (deltas overwrite the consumed activations): delta3 -> H3, delta2 -> H2, delta1 -> H1
    HIPCHK(gemm(D4, n4, nullptr, 0, w.B4, R, n3, WIDE_EPI_BWD, nullptr, nullptr, D3, n3, H3, nullptr, "sdf_wide_gemm"));
    HIPCHK(gemm(H3, n3, nullptr, 0, w.B3h, R, n2, WIDE_EPI_BWD, nullptr, nullptr, D2, n2, H2, nullptr, "sdf_wide_gemm"));
    if (w.e3)
        HIPCHK(gemm(H3, n3, nullptr, 0, w.B3e, R, NEB, WIDE_EPI_STORE, nullptr, nullptr, nullptr, 0, GE3, nullptr,
                    "sdf_wide_gemm"));
    else  // res 'latent': layer 3 does not see the embedding
        HIPCHK(hipMemsetAsync(GE3, 0, (size_t)R * NEB * sizeof(float), st));
    HIPCHK(gemm(H2, n2, nullptr, 0, w.B2, R, n1, WIDE_EPI_BWD, nullptr, nullptr, D1, n1, H1, nullptr, "sdf_wide_gemm"));
    HIPCHK(gemm(H1, n1, nullptr, 0, w.B1e, R, NEB, WIDE_EPI_STORE, nullptr, nullptr, nullptr, 0, GE1, nullptr,
                "sdf_wide_gemm"));
    if (glat) {  // d df / d z = delta1 W1z + delta3 W3z: one GEMM over the two K segments [delta1 | delta3]
        HIPCHK(gemm(H1, n1, H3, n3, w.Bz, R, LZ, WIDE_EPI_STORE, nullptr, nullptr, nullptr, 0, gz, nullptr,
                    "sdf_wide_gemm"));
        if (zpad)
            HIPCHK(hipMemcpy2DAsync(glat, (size_t)LH * sizeof(float), gz, (size_t)LZ * sizeof(float),
                                    (size_t)LH * sizeof(float), (size_t)R, hipMemcpyDeviceToDevice, st));
    }
    ea.H4 = H4; ea.GE3 = GE3; ea.GE1 = GE1; ea.w5 = w.w5; ea.b5 = net->args.b5; ea.out = out4;
    HIPCHK(timed(ctx, "sdf_wide_final", [&] { return launch_wide_final(ea, st); }));
    return SDFNMPC_OK;
}

template <typename T>
static int run_hoist(sdfnmpc_ctx* ctx, const sdfnmpc_net* net, const T* latent, long long stride, int n_inst,
                     float* c13) {
    HoistArgs<T> h{latent, stride, net->WzT, net->bias13, c13, n_inst};
    HIPCHK(timed(ctx, "sdf_hoist", [&] { return launch_hoist<T>(h, ctx->stream); }));
    return SDFNMPC_OK;
}

extern "C" int sdfnmpc_sdf_eval(sdfnmpc_ctx* ctx, const sdfnmpc_net* net, long long rows, const float* pos4,
                                const float* latent, int rows_per_inst, float* out4, float* grad_latent) {
    if (!ctx || !net || (!pos4 && rows > 0) || (!latent && rows > 0) || (!out4 && rows > 0) || rows < 0 ||
        rows_per_inst < 1)
        return fail(SDFNMPC_E_ARG, "bad sdfnmpc_sdf_eval arguments");
    if (net->device != ctx->device) return fail(SDFNMPC_E_ARG, "net and ctx are on different devices");
    if (rows == 0) return SDFNMPC_OK;
    ScopedDevice sd(ctx->device);
    const int n_inst = (int)((rows + rows_per_inst - 1) / rows_per_inst);
    if (net->wide)
        return run_wide(ctx, net, rows, (const float4*)pos4, latent, nullptr, 0, n_inst, rows_per_inst, (float4*)out4,
                        nullptr, grad_latent);
    HIPCHK(ctx->c13.ensure((size_t)n_inst * C13_STRIDE * sizeof(float)));
    int rc = run_hoist<float>(ctx, net, latent, L, n_inst, (float*)ctx->c13.p);
    if (rc) return rc;
    return run_sdf(ctx, net, rows, (const float4*)pos4, (const float*)ctx->c13.p, rows_per_inst, (float4*)out4,
                   grad_latent, grad_latent ? 32 : ctx->tile_rows);
}

// the host-pointer path's wait for its results (polling hipStreamQuery instead measured 3 us slower per
// call; tools/launch_lat.hip: a bare launch + hipStreamSynchronize is 11 us on the box)
static hipError_t host_wait(sdfnmpc_ctx* ctx) { return hipStreamSynchronize(ctx->stream); }

static bool srv_enabled(sdfnmpc_ctx* ctx) {
    if (ctx->srv.mode < 0) {
        const char* e = getenv("SDFNMPC_SDF_SERVER");
        ctx->srv.mode = (e && *e == '0') ? 0 : 1;
        if (const char* ms = getenv("SDFNMPC_SDF_SERVER_IDLE_MS")) {
            const double v = atof(ms);
            if (v > 0.0) ctx->srv.idle_s = v * 1e-3;
        }
        if (const char* ms = getenv("SDFNMPC_SDF_SERVER_LIFE_MS")) {
            const double v = atof(ms);
            if (v > 0.0) ctx->srv.life_s = v * 1e-3;
        }
    }
    return ctx->srv.mode == 1 && !ctx->srv.abandoned;
}

// One request to the resident SDF server (sdf_row.hip): the staged fp32 request (hp [rows][4], hl
// [rows][L]) goes into the mailbox, the results come back into ho in the staged path's layout.  The
// server is (re)launched when it is not running -- first call, a different network, or after it left on
// its idle timeout or its life bound (1 ms and 0.8 ms by default: the longest a device-wide synchronisation
// elsewhere in the process waits for it); a server that exits while a request is posted writes its epoch
// to `gone`, and the caller relaunches at once (the new server serves every seq_in above the seq_out it
// finds).
constexpr int SRV_FALLBACK = 1;  // srv_call: the server was abandoned; the caller takes the per-call launch path
static int srv_call(sdfnmpc_ctx* ctx, const sdfnmpc_net* net, int rows, const float* hp, const float* hl, bool grad,
                    float* ho) {
    using clk = std::chrono::steady_clock;
    auto& S = ctx->srv;
    if (!S.mb) {
        HIPCHK(hipHostMalloc((void**)&S.mb, sizeof(SdfMbox), hipHostMallocCoherent | hipHostMallocMapped));
        memset((void*)S.mb, 0, sizeof(SdfMbox));
        HIPCHK(hipHostGetDevicePointer((void**)&S.mb_dev, S.mb, 0));
        int lo = 0, hi = 0;
        (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
        HIPCHK(hipStreamCreateWithPriority(&S.stream, hipStreamNonBlocking, hi));
        int khz = 0;
        HIPCHK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx->device));
        if (khz <= 0) khz = 100000;
        S.khz = khz;
        S.idle_ticks = (long long)(S.idle_s * khz * 1e3);
        S.life_ticks = (long long)(S.life_s * khz * 1e3);
        S.seq = 0;
        S.live = false;
    }
    if (S.live && S.net != net->uid && !srv_stop(ctx)) return SRV_FALLBACK;  // abandoned: serve this call per launch
    if (S.live && __atomic_load_n(&S.mb->gone, __ATOMIC_ACQUIRE) == S.epoch) {
        // it left (idle, life or stop) after publishing its last answer: nothing of it runs any more but
        // its kernel's exit, which the stream orders before the relaunch
        S.live = false;
        __atomic_store_n(&S.mb->stop, 0ull, __ATOMIC_RELEASE);
    }
    if (S.live && (S.mb->stop || std::chrono::duration<double>(clk::now() - S.last).count() > 0.5 * S.idle_s)) {
        const hipError_t q = hipStreamQuery(S.stream);
        if (q == hipSuccess) {
            S.live = false;
            __atomic_store_n(&S.mb->stop, 0ull, __ATOMIC_RELEASE);
        } else if (q == hipErrorNotReady && S.mb->stop) {
            return fail(SDFNMPC_E_HIP, "sdf server: the previous server has not left yet");
        } else if (q != hipErrorNotReady) {
            return fail(SDFNMPC_E_HIP, std::string("sdf server: ") + hipGetErrorString(q));
        }
    }
    const int LH = net->host.L;  // the mailbox holds [rows][4] | [rows][LH] (SdfMbox)
    memcpy(S.mb->in, hp, (size_t)rows * 4 * sizeof(float));
    memcpy(S.mb->in + (size_t)rows * 4, hl, (size_t)rows * LH * sizeof(float));
    S.mb->rows = rows;
    S.mb->grad = grad ? 1 : 0;
    const unsigned long long seq = ++S.seq;
    __atomic_store_n(&S.mb->seq_in, seq, __ATOMIC_RELEASE);
    auto relaunch = [&]() {
        ++S.epoch;
        return net->wide ? launch_sdf_server_wide(net->wrow, S.mb_dev, S.idle_ticks, S.life_ticks, S.epoch, S.stream)
                         : launch_sdf_server(net->row, S.mb_dev, S.idle_ticks, S.life_ticks, S.epoch, S.stream);
    };
    if (!S.live) {
        HIPCHK(relaunch());
        S.live = true;
        S.net = net->uid;
    }
    const auto t0 = clk::now();
    for (unsigned long spin = 1;; ++spin) {
        if (__atomic_load_n(&S.mb->seq_out, __ATOMIC_ACQUIRE) == seq) break;
        if (__atomic_load_n(&S.mb->gone, __ATOMIC_ACQUIRE) == S.epoch) {
            // the server left between requests (idle / life) without seeing this one: relaunch now
            if (__atomic_load_n(&S.mb->seq_out, __ATOMIC_ACQUIRE) == seq) break;
            HIPCHK(relaunch());
            continue;
        }
        if ((spin & 1023) == 0) {
            const hipError_t q = hipStreamQuery(S.stream);
            if (q == hipSuccess) {  // the server left before it saw this request
                if (__atomic_load_n(&S.mb->seq_out, __ATOMIC_ACQUIRE) == seq) break;
                HIPCHK(relaunch());
            } else if (q != hipErrorNotReady) {
                S.live = false;
                return fail(SDFNMPC_E_HIP, std::string("sdf server: ") + hipGetErrorString(q));
            }
            if (std::chrono::duration<double>(clk::now() - t0).count() > 5.0) {
                // ask it to leave, but do not wait on a server that stopped answering; a later call
                // queries the stream and relaunches only once it has gone
                __atomic_store_n(&S.mb->stop, 1ull, __ATOMIC_RELEASE);
                return fail(SDFNMPC_E_HIP, "sdf server: no answer within 5 s");
            }
        }
    }
    const volatile float* o = S.mb->out;
    const size_t n = (size_t)rows * (grad ? 4 + LH : 4);
    for (size_t i = 0; i < n; ++i) ho[i] = o[i];
    S.last = clk::now();
    const volatile SdfMbox* vm = S.mb;
    S.acc[0] += (double)(vm->t_staged - vm->t_seen) * 1e3 / S.khz;
    S.acc[1] += (double)(vm->t_done - vm->t_staged) * 1e3 / S.khz;
    S.acc[2] += std::chrono::duration<double>(S.last - t0).count() * 1e6;
    S.acc[3] += 1.0;
    if (!net->wide)  // row_eval's phase stamps (the variant server keeps none)
        for (int i = 0; i < 14; ++i)
            S.ph[i] += (double)(vm->t_phase[i] - (i ? vm->t_phase[i - 1] : vm->t_staged)) * 1e3 / S.khz;
    return SDFNMPC_OK;
}

// mean microseconds per served request since the last call: [0] staging the request into LDS, [1] the
// evaluation, [2] the host's wait from posting to the answer; [3] requests; [4..17] the evaluation's
// phases (row_eval's ROW_STAMPs) (diagnostics, tools/c2_server_probe.py)
extern "C" int sdfnmpc_ctx_sdf_server_stats(sdfnmpc_ctx* ctx, double* out18) {
    if (!ctx || !out18) return fail(SDFNMPC_E_ARG, "bad sdfnmpc_ctx_sdf_server_stats arguments");
    std::lock_guard<std::mutex> lk(ctx->mu);
    const double n = ctx->srv.acc[3];
    for (int i = 0; i < 3; ++i) out18[i] = n > 0 ? ctx->srv.acc[i] / n : 0.0;
    out18[3] = n;
    for (int i = 0; i < 14; ++i) out18[4 + i] = n > 0 ? ctx->srv.ph[i] / n : 0.0;
    for (double& a : ctx->srv.acc) a = 0.0;
    for (double& a : ctx->srv.ph) a = 0.0;
    return SDFNMPC_OK;
}

extern "C" int sdfnmpc_ctx_set_sdf_server(sdfnmpc_ctx* ctx, int on) {
    if (!ctx || on < 0 || on > 1) return fail(SDFNMPC_E_ARG, "bad sdfnmpc_ctx_set_sdf_server arguments");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ScopedDevice sd(ctx->device);
    if (!on && !srv_stop(ctx)) return SDFNMPC_E_HIP;
    ctx->srv.mode = on;
    return SDFNMPC_OK;
}

extern "C" int sdfnmpc_sdf_eval_host(sdfnmpc_ctx* ctx, const sdfnmpc_net* net, int rows, const double* in,
                                     double* df, double* grad) {
    if (!ctx || !net || rows < 0 || (rows > 0 && (!in || !df))) return fail(SDFNMPC_E_ARG, "bad sdf_eval_host arguments");
    if (rows == 0) return SDFNMPC_OK;
    std::lock_guard<std::mutex> lk(ctx->mu);
    ScopedDevice sd(ctx->device);
    const int L = net->host.L, D = 3 + L;  // 131 for the deployed net (and every 128-latent one)
    // pinned staging: in [rows][4] pos | [rows][L] latent, out [rows][4] (df, d/dpos) | [rows][L] d/dlatent
    // (double -> float as L4CasADi does); one copy each way, one synchronisation
    const size_t nin = (size_t)rows * (4 + L), bytes = 2 * nin * sizeof(float);
    if (bytes > ctx->h_pin_bytes) {
        if (ctx->h_pin) (void)hipHostFree(ctx->h_pin);
        ctx->h_pin = nullptr;
        ctx->h_pin_bytes = 0;
        HIPCHK(hipHostMalloc((void**)&ctx->h_pin, bytes, hipHostMallocDefault));
        ctx->h_pin_bytes = bytes;
    }
    float* hp = ctx->h_pin;
    float* hl = hp + (size_t)rows * 4;
    float* ho = ctx->h_pin + nin;
    for (int r = 0; r < rows; ++r) {
        for (int c = 0; c < 3; ++c) hp[r * 4 + c] = (float)in[(size_t)r * D + c];
        hp[r * 4 + 3] = 0.0f;
        for (int k = 0; k < L; ++k) hl[(size_t)r * L + k] = (float)in[(size_t)r * D + 3 + k];
    }
    // the row evaluators: sdf_row.hip for the deployed network, sdf_row_wide.hip for a variant that fits it
    const bool use_row = net->wide ? net->wrow_ok && rows <= wide_row_max_rows(L) : rows <= SDF_ROW_MAX;
    bool served = false;
    if (use_row && srv_enabled(ctx)) {  // the resident server: no launch, no copies, no synchronisation
        const int rc = srv_call(ctx, net, rows, hp, hl, grad != nullptr, ho);
        if (rc != SDFNMPC_OK && rc != SRV_FALLBACK) return rc;
        served = rc == SDFNMPC_OK;
    }
    if (!served && use_row) {  // the latency path: one launch, no hoist (sdf_row.hip).  Zero-copy (the kernel reading
        // and writing the pinned block over PCIe) was measured equal in wall time: the PCIe reads add
        // ~2 us to the kernel, as much as the two staging copies cost.
        HIPCHK(ctx->hin.ensure(nin * sizeof(float)));
        HIPCHK(ctx->hout.ensure(nin * sizeof(float)));
        float* dpos = (float*)ctx->hin.p;
        float* dout = (float*)ctx->hout.p;
        HIPCHK(hipMemcpyAsync(dpos, hp, nin * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
        if (net->wide) {
            WideRowArgs ra = net->wrow;
            ra.pos = (const float4*)dpos;
            ra.latent = dpos + (size_t)rows * 4;
            ra.out = (float4*)dout;
            ra.grad_latent = grad ? dout + (size_t)rows * 4 : nullptr;
            ra.rows = rows;
            HIPCHK(timed(ctx, "sdf_row_wide", [&] { return launch_sdf_row_wide(ra, ctx->stream); }));
        } else {
            SdfRowArgs ra = net->row;
            ra.pos = (const float4*)dpos;
            ra.latent = dpos + (size_t)rows * 4;
            ra.out = (float4*)dout;
            ra.grad_latent = grad ? dout + (size_t)rows * 4 : nullptr;
            ra.rows = rows;
            HIPCHK(timed(ctx, "sdf_row", [&] { return launch_sdf_row(ra, ctx->stream); }));
        }
        HIPCHK(hipMemcpyAsync(ho, dout, (grad ? nin : (size_t)rows * 4) * sizeof(float), hipMemcpyDeviceToHost,
                              ctx->stream));
        HIPCHK(host_wait(ctx));
    } else if (!served) {
        HIPCHK(ctx->hin.ensure(nin * sizeof(float)));
        HIPCHK(ctx->hout.ensure(nin * sizeof(float)));
        float* dpos = (float*)ctx->hin.p;
        float* dlat = dpos + (size_t)rows * 4;
        float* dout = (float*)ctx->hout.p;
        float* dglat = dout + (size_t)rows * 4;
        // the latent hoist depends on the latents only: reuse it while they repeat (the same image's
        // latent at every shooting node of an RTI); the positions go up every call
        const bool same_lat = !net->wide && ctx->h_net == net->uid && ctx->h_lat.size() == (size_t)rows * L &&
                              !memcmp(ctx->h_lat.data(), hl, (size_t)rows * L * sizeof(float));
        HIPCHK(hipMemcpyAsync(dpos, hp, (same_lat ? (size_t)rows * 4 : nin) * sizeof(float), hipMemcpyHostToDevice,
                              ctx->stream));
        int rc = SDFNMPC_OK;
        if (net->wide) {
            rc = sdfnmpc_sdf_eval(ctx, net, rows, dpos, dlat, 1, dout, grad ? dglat : nullptr);
        } else {
            if (!same_lat) {
                HIPCHK(ctx->hc13.ensure((size_t)rows * C13_STRIDE * sizeof(float)));
                rc = run_hoist<float>(ctx, net, dlat, L, rows, (float*)ctx->hc13.p);
                if (rc) return rc;
                ctx->h_lat.assign(hl, hl + (size_t)rows * L);
                ctx->h_net = net->uid;
            }
            rc = run_sdf(ctx, net, rows, (const float4*)dpos, (const float*)ctx->hc13.p, 1, (float4*)dout,
                         grad ? dglat : nullptr, grad ? 32 : ctx->tile_rows);
        }
        if (rc) {
            ctx->h_net = 0;
            return rc;
        }
        HIPCHK(hipMemcpyAsync(ho, dout, (grad ? nin : (size_t)rows * 4) * sizeof(float), hipMemcpyDeviceToHost,
                              ctx->stream));
        HIPCHK(host_wait(ctx));
    }
    const float* go = ho + (size_t)rows * 4;
    for (int r = 0; r < rows; ++r) {
        df[r] = ho[(size_t)r * 4];
        if (grad) {
            for (int c = 0; c < 3; ++c) grad[(size_t)r * D + c] = ho[(size_t)r * 4 + 1 + c];
            for (int k = 0; k < L; ++k) grad[(size_t)r * D + 3 + k] = go[(size_t)r * L + k];
        }
    }
    return SDFNMPC_OK;
}

// ------------------------------------------------------------------------------------------------
// batched preparation phase
// pk != NULL (sdfnmpc_rti_prepare): the QP stage records are packed in the same phase.  With ny == 11
// the pack runs after the linearisation on the aux stream, beside the SDF kernel, and only the sdf row
// of C^T waits for the join; with the sdf cost (ny == 12) H and g depend on h[2], so the whole pack
// follows the join.
static int lin_impl(sdfnmpc_ctx* ctx, const sdfnmpc_net* net, const sdfnmpc_quad_model* mdl,
                    const sdfnmpc_lin_args* a, const QpArgs* pk, bool* split_out = nullptr) {
    if (!ctx || !mdl || !a) return fail(SDFNMPC_E_ARG, "NULL argument");
    const bool no_sdf = a->no_sdf != 0;
    if (!net && !no_sdf) return fail(SDFNMPC_E_ARG, "NULL network (only allowed with lin_args.no_sdf)");
    if (a->B < 0 || a->N < 1 || a->np < 17 + (net ? net->host.L : 0) || (a->latent_mode != 0 && a->latent_mode != 1))
        return fail(SDFNMPC_E_ARG, "bad B/N/np/latent_mode");
    const int nyN = a->nyN == 0 ? 4 : a->nyN;
    if (nyN != 4 && nyN != 5) return fail(SDFNMPC_E_ARG, "lin_args.nyN must be 4 or 5");
    if ((nyN == 5) != (mdl->stability != 0)) return fail(SDFNMPC_E_ARG, "nyN == 5 exactly with model.stability");
    if (mdl->rec_feas && (mdl->poly_deg < 0 || mdl->poly_deg > SDFNMPC_POLY_DEG_MAX))
        return fail(SDFNMPC_E_ARG, "model.poly_deg must be 0..6");
    if ((mdl->rec_feas || mdl->stability) && (!a->hE || !a->JhE))
        return fail(SDFNMPC_E_ARG, "rec_feas / stability need lin_args.hE and JhE");
    if (a->B == 0) return SDFNMPC_OK;
    if (!a->x || !a->u || !a->p || !a->dt || !a->xn || !a->AB || !a->y || !a->Jy || !a->yN || !a->JyN || !a->h ||
        !a->Jh)
        return fail(SDFNMPC_E_ARG, "NULL array in sdfnmpc_lin_args");
    if (net && net->device != ctx->device) return fail(SDFNMPC_E_ARG, "net and ctx are on different devices");
    ScopedDevice sd(ctx->device);
    const long long rows = (long long)a->B * (a->N + 1);
    float4* sdf4 = (float4*)a->sdf;
    if (!sdf4) {
        HIPCHK(ctx->sdf4.ensure((size_t)rows * 16));
        sdf4 = (float4*)ctx->sdf4.p;
    }
    const int n_inst = a->latent_mode == 0 ? a->B : (int)rows;
    if (!no_sdf && !net->wide) HIPCHK(ctx->c13.ensure((size_t)n_inst * C13_STRIDE * sizeof(float)));
    // dynamics / cost / FOV constraints (independent of the network): forked onto the low-priority
    // aux stream so they fill the CUs the SDF kernel leaves idle (its tail), joined at the end
    LinArgs la{};
    la.x = a->x; la.u = a->u; la.p = a->p; la.dt = a->dt;
    la.xn = a->xn; la.AB = a->AB; la.y = a->y; la.Jy = a->Jy; la.yN = a->yN; la.JyN = a->JyN; la.h = a->h; la.Jh = a->Jh;
    la.B = a->B; la.N = a->N; la.np = a->np;
    la.m.gamma = mdl->gamma; la.m.roll = mdl->roll; la.m.pitch = mdl->pitch; la.m.wz = mdl->wz; la.m.g = mdl->g;
    for (int i = 0; i < 3; ++i)  // B_R_C^T B_p_C + [fov_const_offset, 0, 0]
        la.m.fov_off[i] = mdl->B_R_C[0 * 3 + i] * mdl->B_p_C[0] + mdl->B_R_C[1 * 3 + i] * mdl->B_p_C[1] +
                          mdl->B_R_C[2 * 3 + i] * mdl->B_p_C[2] + (i == 0 ? mdl->fov_const_offset : 0.0);
    la.m.max_df = net ? net->host.max_df : 1.0;
    for (int i = 0; i < 9; ++i) la.m.B_R_C[i] = mdl->B_R_C[i];
    la.m.rec_feas = mdl->rec_feas ? 1 : 0;
    la.m.stability = mdl->stability ? 1 : 0;
    la.m.poly_deg = mdl->poly_deg;
    for (int i = 0; i < SDFNMPC_POLY_MAX; ++i) la.m.poly[i] = mdl->poly[i];
    la.hE = a->hE;
    la.JhE = a->JhE;
    la.nyN = nyN;
    QpArgs pa{};
    // serial: the linearisation (and the whole pack) after the SDF kernel on the one stream -- the diagnostic
    // SDFNMPC_SERIAL_PREP, and the few-row latency path (B = 1), where the fork / join's event waits cost
    // more than the overlap gains (round 5: 0.643 vs 0.646 ms per B = 1 step)
    const bool serial = ctx->serial_prep || (!no_sdf && !net->wide && rows <= SDF_ROW_PREP_MAX);
    const bool split = pk && pk->ny == 11 && !serial && !no_sdf;  // pack beside the SDF kernel
    if (split_out) *split_out = split;
    if (pk) {
        pa = *pk;
        pa.pack_part = split ? 1 : 0;
    }
    // the fork: ev_fork marks the main stream's state (the inputs written), the auxiliary stream waits for
    // it and runs the linearisation (+ the pack's first part) beside the SDF kernel
    auto fork_mark = [&]() -> int {
        if (serial) return SDFNMPC_OK;
        HIPCHK(hipEventRecord(ctx->ev_fork, ctx->stream));
        return SDFNMPC_OK;
    };
    auto fork_launch = [&]() -> int {
        if (serial) return SDFNMPC_OK;
        HIPCHK(hipStreamWaitEvent(ctx->aux, ctx->ev_fork, 0));
        HIPCHK(timed(ctx, "linearize", [&] { return launch_linearize(la, ctx->aux); }, ctx->aux));
        if (split) HIPCHK(timed(ctx, "rti_qp_pack", [&] { return launch_rti_qp_pack(pa, ctx->aux); }, ctx->aux));
        HIPCHK(hipEventRecord(ctx->ev_join, ctx->aux));
        return SDFNMPC_OK;
    };
    auto fork_lin = [&]() -> int {
        int rc_ = fork_mark();
        return rc_ ? rc_ : fork_launch();
    };
    // after the join: the rest of the pack on the main stream
    auto finish_pack = [&]() -> int {
        if (!pk) return SDFNMPC_OK;
        // split: the sdf row of C^T is copied by rti_qp_kernel itself (sdf_row_patch), no launch here
        if (!split) HIPCHK(timed(ctx, "rti_qp_pack", [&] { return launch_rti_qp_pack(pa, ctx->stream); }));
        return SDFNMPC_OK;
    };
    int rc;
    if (no_sdf) {  // no constraint or cost reads the network: the linearisation alone, then the pack
        HIPCHK(timed(ctx, "linearize", [&] { return launch_linearize(la, ctx->stream); }, ctx->stream));
        return finish_pack();
    }
    if (ctx->lin_first && (rc = fork_lin())) return rc;
    // 2. latent hoisting (latent = p[.][17:] as fp32)
    const long long stride = a->latent_mode == 0 ? (long long)(a->N + 1) * a->np : (long long)a->np;
    SdfArgs cons{};
    cons.x = a->x;
    cons.p = a->p;
    cons.np = a->np;
    cons.h = a->h;
    cons.Jh = a->Jh;
    cons.max_df = net->host.max_df;
    if (net->wide) {  // layer-by-layer schedule, linearisation forked first so it overlaps the GEMMs
        if (!ctx->lin_first && (rc = fork_lin())) return rc;
        rc = run_wide(ctx, net, rows, nullptr, nullptr, a->p + 17, stride, n_inst, a->latent_mode == 0 ? a->N + 1 : 1,
                      sdf4, &cons);
        if (rc) return rc;
        if (serial) {
            HIPCHK(timed(ctx, "linearize", [&] { return launch_linearize(la, ctx->stream); }, ctx->stream));
            return finish_pack();
        }
        HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->ev_join, 0));
        return finish_pack();
    }
    if (rows <= SDF_ROW_PREP_MAX) {  // a few rows (B = 1): one workgroup per row, no hoist
        // the row kernel is the critical path: queued right after the fork mark, before the host spends
        // the auxiliary stream's API calls (≈15 µs at B = 1, round 5 trace), which the mark keeps it
        // independent of
        if (!ctx->lin_first && (rc = fork_mark())) return rc;
        SdfRowArgs ra = net->row;
        ra.x = a->x; ra.p = a->p; ra.np = a->np;
        ra.zd = a->p + 17; ra.zstride = stride; ra.rows_per_inst = a->latent_mode == 0 ? a->N + 1 : 1;
        ra.h = a->h; ra.Jh = a->Jh; ra.max_df = net->host.max_df;
        ra.out = sdf4;
        ra.rows = (int)rows;
        HIPCHK(timed(ctx, "sdf_row", [&] { return launch_sdf_row(ra, ctx->stream); }));
        if (!ctx->lin_first && (rc = fork_launch())) return rc;
    } else {
        rc = run_hoist<double>(ctx, net, a->p + 17, stride, n_inst, (float*)ctx->c13.p);
        if (rc) return rc;
        if (!ctx->lin_first && (rc = fork_lin())) return rc;
        // 3. network forward + position gradient, with the sdf row of h / J_h in its epilogue
        rc = run_sdf(ctx, net, rows, nullptr, (const float*)ctx->c13.p,
                     a->latent_mode == 0 ? a->N + 1 : 1, sdf4, nullptr, ctx->tile_rows, &cons);
        if (rc) return rc;
    }
    if (serial) {
        HIPCHK(timed(ctx, "linearize", [&] { return launch_linearize(la, ctx->stream); }, ctx->stream));
        return finish_pack();
    }
    HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->ev_join, 0));
    return finish_pack();
}

extern "C" int sdfnmpc_linearize(sdfnmpc_ctx* ctx, const sdfnmpc_net* net, const sdfnmpc_quad_model* mdl,
                                 const sdfnmpc_lin_args* a) {
    if (ctx) ctx->prep.valid = false;  // lin outputs may change under records packed earlier
    return lin_impl(ctx, net, mdl, a, nullptr);
}

// ------------------------------------------------------------------------------------------------
// batched QP (feedback phase) and RTI step
// the constraint set of sdfnmpc_qp_opts (include/sdfnmpc.h): counts, columns and their order
static int qp_cset_check(const sdfnmpc_qp_opts* o) {
    if (o->nh < 0 || o->nh > 3) return fail(SDFNMPC_E_ARG, "qp opts: nh must be 0..3");
    for (int j = 0; j < o->nh; ++j)
        if (o->h_col[j] < 0 || o->h_col[j] > 2 || (j && o->h_col[j] == o->h_col[0]) || (j == 2 && o->h_col[2] == o->h_col[1]))
            return fail(SDFNMPC_E_ARG, "qp opts: h_col must be distinct columns 0..2");
    if (o->nhs < 0 || o->nhs > o->nh) return fail(SDFNMPC_E_ARG, "qp opts: nhs (hard stage rows) must be 0..nh");
    if (o->nhN < 0 || o->nhN > SDFNMPC_NHN_MAX || o->nsN < 0 || o->nsN > 3 || o->nsN > o->nhN || o->nhN - o->nsN > 6)
        return fail(SDFNMPC_E_ARG, "qp opts: terminal rows nhN <= 8 with nsN <= 3 soft and <= 6 hard");
    for (int j = 0; j < o->nhN; ++j) {
        if (o->hN_col[j] < -1 || o->hN_col[j] > 2 || o->hE_col[j] < -1 || o->hE_col[j] >= SDFNMPC_NHE ||
            (o->hN_col[j] < 0 && o->hE_col[j] < 0))
            return fail(SDFNMPC_E_ARG, "qp opts: terminal row j needs hN_col in -1..2 / hE_col in -1..5, not both -1");
        if (!(o->lhN[j] <= o->uhN[j])) return fail(SDFNMPC_E_ARG, "qp opts: terminal bounds lhN > uhN");
    }
    if (o->nyN != 4 && o->nyN != 5) return fail(SDFNMPC_E_ARG, "qp opts: nyN must be 4 or 5");
    return SDFNMPC_OK;
}
static QpRows qp_rows_of(const sdfnmpc_qp_opts* o) { return QpRows{o->nh, o->nhN, o->nsN, o->nhs}; }
// the network is read by a constraint row (stage h_col or terminal hN_col == 2) or the sdf cost
static bool qp_needs_sdf(const sdfnmpc_qp_opts* o) {
    bool need = o->ny == 12;
    for (int j = 0; j < o->nh; ++j) need = need || o->h_col[j] == 2;
    for (int j = 0; j < o->nhN; ++j) need = need || o->hN_col[j] == 2;
    return need;
}
// validation and kernel arguments shared by sdfnmpc_qp_solve / sdfnmpc_rti_prepare / sdfnmpc_qp_feedback
// (sizes the workspace; the caller holds the device scope)
static int qp_build(sdfnmpc_ctx* ctx, const sdfnmpc_qp_opts* o, const sdfnmpc_qp_args* a, QpArgs& q) {
    if (a->B < 0 || a->N < 1 || a->N > 200) return fail(SDFNMPC_E_ARG, "bad B/N for the QP");
    if (!a->xn || !a->AB || !a->y || !a->Jy || !a->yN || !a->JyN || !a->h || !a->Jh || !a->x || !a->u || !a->x0 ||
        !a->yref || !a->W || !a->yNref || !a->WN || !a->dt || !a->dx || !a->du)
        return fail(SDFNMPC_E_ARG, "NULL array in sdfnmpc_qp_args");
    if (o->lm <= 0.0 || o->max_iter < 1 || !(o->tol > 0.0))
        return fail(SDFNMPC_E_ARG, "qp opts: lm > 0 (strict convexity), max_iter >= 1, tol > 0 required");
    if (o->ny != 11 && o->ny != 12) return fail(SDFNMPC_E_ARG, "qp opts: ny must be 11 or 12 (sdf_cost)");
    if (int rc = qp_cset_check(o)) return rc;
    bool term_e = false;
    for (int j = 0; j < o->nhN; ++j) term_e = term_e || o->hE_col[j] >= 0;
    if (term_e && (!a->hE || !a->JhE)) return fail(SDFNMPC_E_ARG, "qp args: terminal rows read hE / JhE (NULL)");
    if (qp_lds_bytes(a->N, qp_rows_of(o)) > ctx->lds_per_cu)
        return fail(SDFNMPC_E_UNSUPPORTED, "horizon too long for the LDS-resident QP");
    HIPCHK(ctx->qpw.ensure((size_t)a->B * qp_work_doubles(a->N) * sizeof(double)));
    const bool own_st = !a->status || !a->iters || !a->res;
    if (own_st) HIPCHK(ctx->qpst.ensure((size_t)a->B * (2 * sizeof(int) + 2 * sizeof(double))));
    q = QpArgs{};
    q.B = a->B; q.N = a->N;
    q.xn = a->xn; q.AB = a->AB; q.y = a->y; q.Jy = a->Jy; q.yN = a->yN; q.JyN = a->JyN; q.h = a->h; q.Jh = a->Jh;
    q.hE = a->hE; q.JhE = a->JhE;
    q.x = a->x; q.u = a->u; q.x0 = a->x0; q.yref = a->yref; q.W = a->W; q.yNref = a->yNref; q.WN = a->WN; q.dt = a->dt;
    q.dx = a->dx; q.du = a->du; q.slack = a->slack;
    double* stbuf = (double*)ctx->qpst.p;
    q.res = a->res ? a->res : stbuf;
    q.status = a->status ? a->status : (int*)(stbuf + 2 * a->B);
    q.iters = a->iters ? a->iters : (int*)(stbuf + 2 * a->B) + a->B;
    q.work = (double*)ctx->qpw.p;
    for (int i = 0; i < 4; ++i) { q.lbu[i] = o->lbu[i]; q.ubu[i] = o->ubu[i]; }
    for (int i = 0; i < 3; ++i) { q.lh[i] = o->lh[i]; q.uh[i] = o->uh[i]; q.zl[i] = o->zl[i]; q.Zl[i] = o->Zl[i]; }
    q.lm = o->lm; q.tol = o->tol; q.max_iter = o->max_iter; q.cost_scaling = o->cost_scaling; q.ny = o->ny;
    q.lm_scaling = o->lm_scaling;
    q.warm_start = o->warm_start ? 1 : 0;
    q.nh = o->nh; q.nhN = o->nhN; q.nsN = o->nsN; q.nyN = o->nyN; q.nhs = o->nhs;
    q.seg_rows = qp_is_seg_set(*o) ? 1 : 0;
    q.sdf_row = -1;
    for (int j = 0; j < 3; ++j) {
        q.h_col[j] = j < o->nh ? o->h_col[j] : 0;
        if (j < o->nh && o->h_col[j] == 2) q.sdf_row = j;
        q.zlN[j] = o->zlN[j]; q.ZlN[j] = o->ZlN[j];
    }
    for (int j = 0; j < QP_NHN; ++j) {
        q.hN_col[j] = j < o->nhN ? o->hN_col[j] : -1;
        q.hE_col[j] = j < o->nhN ? o->hE_col[j] : -1;
        q.lhN[j] = o->lhN[j]; q.uhN[j] = o->uhN[j];
    }
    return SDFNMPC_OK;
}

// the constraint set a preparation packed its records under (stage rows' columns and kinds, terminal rows'
// columns, the terminal residual width) and the feedback must match: an FNV-1a hash of those fields
static long long cset_key(const QpArgs& q) {
    unsigned long long h = 1469598103934665603ull;
    auto mix = [&](long long v) { h = (h ^ (unsigned long long)(v + 7)) * 1099511628211ull; };
    mix(q.nh); mix(q.nhs); mix(q.nhN); mix(q.nsN); mix(q.nyN);
    for (int j = 0; j < 3; ++j) mix(q.h_col[j]);
    for (int j = 0; j < QP_NHN; ++j) { mix(q.hN_col[j]); mix(q.hE_col[j]); }
    return (long long)(h >> 1);
}

// the IPM kernel of this context and horizon: the segmented one (four wavefronts per instance,
// rti_qp_seg.hip) where it supports N, unless the context asks for the serial one (rti_qp.hip)
static hipError_t qp_launch(sdfnmpc_ctx* ctx, const QpArgs& q) {
    if (qp_kernel_for(ctx, q.N, q.B, q.seg_rows != 0) == SDFNMPC_QP_SEGMENTED) return launch_rti_qp_seg(q, ctx->stream);
    return launch_rti_qp(q, ctx->stream);
}

extern "C" int sdfnmpc_qp_solve(sdfnmpc_ctx* ctx, const sdfnmpc_qp_opts* o, const sdfnmpc_qp_args* a) {
    if (!ctx || !o || !a) return fail(SDFNMPC_E_ARG, "NULL argument");
    ctx->prep.valid = false;  // the workspace is repacked here
    if (a->B == 0) return SDFNMPC_OK;
    ScopedDevice sd(ctx->device);
    QpArgs q;
    if (int rc = qp_build(ctx, o, a, q)) return rc;
    HIPCHK(timed(ctx, "rti_qp_pack", [&] { return launch_rti_qp_pack(q, ctx->stream); }));
    HIPCHK(timed(ctx, "rti_qp", [&] { return qp_launch(ctx, q); }));
    return SDFNMPC_OK;
}

extern "C" int sdfnmpc_rti_prepare(sdfnmpc_ctx* ctx, const sdfnmpc_net* net, const sdfnmpc_quad_model* mdl,
                                   const sdfnmpc_lin_args* la, const sdfnmpc_qp_opts* o, const sdfnmpc_qp_args* qa) {
    if (!ctx || !mdl || !la || !o || !qa) return fail(SDFNMPC_E_ARG, "NULL argument");
    if (la->no_sdf && qp_needs_sdf(o)) return fail(SDFNMPC_E_ARG, "rti_prepare: lin_args.no_sdf, but the QP reads the sdf");
    if ((la->nyN == 0 ? 4 : la->nyN) != o->nyN) return fail(SDFNMPC_E_ARG, "rti_prepare: lin_args.nyN != qp opts nyN");
    ctx->prep.valid = false;
    if (la->B != qa->B || la->N != qa->N) return fail(SDFNMPC_E_ARG, "rti_prepare: lin and qp args differ in B / N");
    if (la->xn != qa->xn || la->AB != qa->AB || la->y != qa->y || la->Jy != qa->Jy || la->yN != qa->yN ||
        la->JyN != qa->JyN || la->h != qa->h || la->Jh != qa->Jh || la->x != qa->x || la->u != qa->u)
        return fail(SDFNMPC_E_ARG, "rti_prepare: the qp args must name the lin args' iterate and outputs");
    if (la->B == 0) return SDFNMPC_OK;
    ScopedDevice sd(ctx->device);
    QpArgs q;
    if (int rc = qp_build(ctx, o, qa, q)) return rc;
    bool split = false;
    if (int rc = lin_impl(ctx, net, mdl, la, &q, &split)) return rc;
    ctx->prep.valid = true;
    ctx->prep.sdf_row_patch = split;  // lin_impl's split pack: no sdf row in the records
    ctx->prep.B = qa->B;
    ctx->prep.N = qa->N;
    ctx->prep.xn = qa->xn;
    ctx->prep.work = q.work;
    ctx->prep.ny = q.ny;
    ctx->prep.lm = q.lm;
    ctx->prep.cost_scaling = q.cost_scaling;
    ctx->prep.lm_scaling = q.lm_scaling;
    ctx->prep.cset = cset_key(q);
    return SDFNMPC_OK;
}

extern "C" int sdfnmpc_qp_feedback(sdfnmpc_ctx* ctx, const sdfnmpc_qp_opts* o, const sdfnmpc_qp_args* a) {
    if (!ctx || !o || !a) return fail(SDFNMPC_E_ARG, "NULL argument");
    if (a->B == 0) return SDFNMPC_OK;
    if (!ctx->prep.valid || ctx->prep.B != a->B || ctx->prep.N != a->N || ctx->prep.xn != a->xn)
        return fail(SDFNMPC_E_ARG, "qp_feedback: no stage records from sdfnmpc_rti_prepare for these arguments");
    ScopedDevice sd(ctx->device);
    QpArgs q;
    if (int rc = qp_build(ctx, o, a, q)) return rc;
    if (q.work != ctx->prep.work) return fail(SDFNMPC_E_ARG, "qp_feedback: workspace moved since rti_prepare");
    if (q.ny != ctx->prep.ny || q.lm != ctx->prep.lm || q.cost_scaling != ctx->prep.cost_scaling ||
        q.lm_scaling != ctx->prep.lm_scaling || cset_key(q) != ctx->prep.cset)  // the stage records hold H, g, C^T
        // packed under the prepare's options
        return fail(SDFNMPC_E_ARG, "qp_feedback: ny / lm / cost scaling / the constraint set differ from sdfnmpc_rti_prepare's");
    ctx->prep.valid = false;  // one feedback per preparation, as in acados' SQP-RTI
    q.sdf_row_patch = ctx->prep.sdf_row_patch ? 1 : 0;
    HIPCHK(timed(ctx, "rti_qp", [&] { return qp_launch(ctx, q); }));
    return SDFNMPC_OK;
}

// ------------------------------------------------------------------------------------------------
// the control step as a HIP graph (include/sdfnmpc.h sdfnmpc_step_create)
struct sdfnmpc_step {
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    int device = 0;
    const sdfnmpc_ctx* ctx = nullptr;  // the context whose workspaces the graph's kernels address
    unsigned long long ws_gen = 0;     // ctx_ws_gen at capture
};
// The graph's kernels hold the context's device workspaces as they were at capture.  Every reallocation
// (a later call with a larger B or N grows them: DevBuf::ensure frees the old buffer) bumps a DevBuf's
// generation, so the sum over the workspaces changes exactly when one of them moved.
static unsigned long long ctx_ws_gen(const sdfnmpc_ctx* c) {
    return c->c13.gen + c->sdf4.gen + c->lat.gen + c->out4.gen + c->glat.gen + c->qpw.gen + c->qpst.gen + c->wws.gen;
}

static int step_eager(sdfnmpc_ctx* ctx, const sdfnmpc_net* net, const sdfnmpc_quad_model* mdl, const sdfnmpc_lin_args* la,
                      const sdfnmpc_qp_opts* o, const sdfnmpc_qp_args* qa, double* u0, const int* status) {
    if (int rc = sdfnmpc_rti_prepare(ctx, net, mdl, la, o, qa)) return rc;
    if (int rc = sdfnmpc_qp_feedback(ctx, o, qa)) return rc;
    // the step applies to the iterate the QP linearised about (qp_args.x, .u: the caller's writable buffers)
    return sdfnmpc_rti_apply(ctx, qa->B, qa->N, const_cast<double*>(qa->x), const_cast<double*>(qa->u), qa->dx, qa->du, u0,
                             status);
}

extern "C" int sdfnmpc_step_create(sdfnmpc_ctx* ctx, const sdfnmpc_net* net, const sdfnmpc_quad_model* mdl,
                                   const sdfnmpc_lin_args* la, const sdfnmpc_qp_opts* o, const sdfnmpc_qp_args* qa,
                                   double* u0, const int* status, sdfnmpc_step** out) {
    if (!ctx || !mdl || !la || !o || !qa || !out) return fail(SDFNMPC_E_ARG, "NULL argument to sdfnmpc_step_create");
    *out = nullptr;
    if (qa->B < 1) return fail(SDFNMPC_E_ARG, "step_create: B must be >= 1");
    // once eagerly: every workspace is allocated and every argument checked before the capture (no
    // allocation may happen inside it)
    if (int rc = step_eager(ctx, net, mdl, la, o, qa, u0, status)) return rc;
    ScopedDevice sd(ctx->device);
    HIPCHK(hipStreamSynchronize(ctx->stream));
    // capture on a private stream (the context stream may be the legacy null stream, which cannot be
    // captured); the fork / join events bring the auxiliary stream into the capture
    hipStream_t cs = nullptr;
    HIPCHK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    hipStream_t saved = ctx->stream;
    const bool timing = ctx->timing;
    ctx->timing = false;
    ctx->stream = cs;
    hipGraph_t g = nullptr;
    int rc = SDFNMPC_OK;
    hipError_t e = hipStreamBeginCapture(cs, hipStreamCaptureModeRelaxed);
    if (e == hipSuccess) {
        rc = step_eager(ctx, net, mdl, la, o, qa, u0, status);
        e = hipStreamEndCapture(cs, &g);  // always ends the capture, also after a failed call
    }
    ctx->stream = saved;
    ctx->timing = timing;
    (void)hipStreamDestroy(cs);
    if (rc) {
        if (g) (void)hipGraphDestroy(g);
        return rc;
    }
    if (e != hipSuccess || !g) {
        if (g) (void)hipGraphDestroy(g);
        return fail(SDFNMPC_E_HIP, std::string("step_create: stream capture failed: ") + hipGetErrorString(e));
    }
    hipGraphExec_t x = nullptr;
    e = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
    if (e != hipSuccess) {
        (void)hipGraphDestroy(g);
        return fail(SDFNMPC_E_HIP, std::string("step_create: graph instantiation failed: ") + hipGetErrorString(e));
    }
    auto* st = new sdfnmpc_step;
    st->graph = g;
    st->exec = x;
    st->device = ctx->device;
    st->ctx = ctx;
    st->ws_gen = ctx_ws_gen(ctx);
    *out = st;
    return SDFNMPC_OK;
}

extern "C" int sdfnmpc_step_launch(sdfnmpc_ctx* ctx, sdfnmpc_step* st) {
    if (!ctx || !st) return fail(SDFNMPC_E_ARG, "NULL argument to sdfnmpc_step_launch");
    if (st->device != ctx->device || st->ctx != ctx) return fail(SDFNMPC_E_ARG, "step_launch: step captured on another context");
    if (ctx_ws_gen(ctx) != st->ws_gen)
        return fail(SDFNMPC_E_ARG, "step_launch: a context workspace was reallocated since the capture (a call with a larger "
                                   "B or N); destroy the step and create it again");
    ScopedDevice sd(ctx->device);
    HIPCHK(hipGraphLaunch(st->exec, ctx->stream));
    return SDFNMPC_OK;
}

extern "C" void sdfnmpc_step_destroy(sdfnmpc_step* st) {
    if (!st) return;
    ScopedDevice sd(st->device);
    if (st->exec) (void)hipGraphExecDestroy(st->exec);
    if (st->graph) (void)hipGraphDestroy(st->graph);
    delete st;
}

extern "C" int sdfnmpc_pack_refs(sdfnmpc_ctx* ctx, const sdfnmpc_ref_opts* o, const sdfnmpc_ref_args* a) {
    if (!ctx || !o || !a) return fail(SDFNMPC_E_ARG, "NULL argument to sdfnmpc_pack_refs");
    if (a->B < 0 || a->N < 1 || a->np < 17 || (a->ny != 11 && a->ny != 12) || !a->p)
        return fail(SDFNMPC_E_ARG, "pack_refs: bad B / N / np / ny or NULL p");
    if (o->mode < -1 || o->mode > 2) return fail(SDFNMPC_E_ARG, "pack_refs: mode must be -1..2");
    if (o->mode >= 0 && (!a->x0 || a->x0_stride < 7 || !a->wrow || !a->yref || !a->W || !a->yNref || !a->WN))
        return fail(SDFNMPC_E_ARG, "pack_refs: x0 (stride >= 7), wrow and the reference outputs are required");
    if (o->mode == 0 && (a->n_wp < 1 || a->n_wp > RP_MAX_WP || !a->wp_p || !a->wp_q))
        return fail(SDFNMPC_E_ARG, "pack_refs: mode 0 needs 1..32 waypoints (wp_p, wp_q)");
    if (o->mode == 1 && !a->vw) return fail(SDFNMPC_E_ARG, "pack_refs: mode 1 needs vw");
    if (a->latent && (!a->W_p_Bo || !a->W_R_Bo || a->L < 1 || 17 + a->L > a->np))
        return fail(SDFNMPC_E_ARG, "pack_refs: latent needs W_p_Bo, W_R_Bo and 17 + L <= np");
    ScopedDevice sd(ctx->device);
    RefPackArgs r{};
    r.B = a->B; r.N = a->N; r.np_ = a->np; r.ny = a->ny; r.n_wp = a->n_wp; r.L = a->L;
    r.nyN = a->nyN == 0 ? 4 : a->nyN;
    if (r.nyN != 4 && r.nyN != 5) return fail(SDFNMPC_E_ARG, "pack_refs: nyN must be 4 or 5");
    r.mode = o->mode; r.yaw_mode = o->yaw_mode; r.st_enable = o->st_enable; r.st_mode = o->st_mode;
    r.st_dang = o->st_dang; r.align_off = o->align_off; r.dmin = o->dmin; r.vref = o->vref; r.wzref = o->wzref;
    r.T = o->T;
    for (int i = 0; i < 3; ++i) r.B_p_C[i] = o->B_p_C[i];
    for (int i = 0; i < 9; ++i) r.B_R_C[i] = o->B_R_C[i];
    r.x0 = a->x0; r.x0_stride = a->x0_stride; r.wp_p = a->wp_p; r.wp_q = a->wp_q; r.vw = a->vw; r.wrow = a->wrow;
    r.latent = a->latent; r.W_p_Bo = a->W_p_Bo; r.W_R_Bo = a->W_R_Bo; r.flag = a->flag;
    r.p = a->p; r.yref = a->yref; r.W = a->W; r.yNref = a->yNref; r.WN = a->WN;
    HIPCHK(timed(ctx, "ref_pack", [&] { return launch_ref_pack(r, ctx->stream); }));
    return SDFNMPC_OK;
}

extern "C" int sdfnmpc_rti_apply(sdfnmpc_ctx* ctx, int B, int N, double* x, double* u, const double* dx,
                                 const double* du, double* u0, const int* status) {
    if (!ctx || B < 0 || N < 1 || (B > 0 && (!x || !u || !dx || !du))) return fail(SDFNMPC_E_ARG, "bad rti_apply arguments");
    ScopedDevice sd(ctx->device);
    HIPCHK(timed(ctx, "rti_apply", [&] { return launch_rti_apply(B, N, x, u, dx, du, u0, status, ctx->stream); }));
    return SDFNMPC_OK;
}

// ------------------------------------------------------------------------------------------------
// shooting grid: numpy.linspace(start, stop, num) = i * ((stop - start) / (num - 1)) + start, last = stop
static void np_linspace(double start, double stop, int num, double* y) {
    if (num == 1) {  // numpy: div = 0 -> y = [start]
        y[0] = start;
        return;
    }
    const double step = (stop - start) / (num - 1);
    for (int i = 0; i < num; ++i) {
        volatile double t = (double)i * step;  // two roundings as numpy, no FMA contraction
        y[i] = t + start;
    }
    if (num > 1) y[num - 1] = stop;
}

extern "C" int sdfnmpc_shooting_grid(int N, double T, int uniform, int n_short, double dt_short, double* nodes,
                                     double* dt) {
    if (N < 1 || !nodes || !dt) return fail(SDFNMPC_E_ARG, "bad grid arguments");
    if (uniform) {
        np_linspace(0.0, T, N + 1, nodes);
    } else {
        if (n_short < 1 || n_short > N) return fail(SDFNMPC_E_ARG, "nb_short_nodes out of range");
        np_linspace(0.0, dt_short * (n_short - 1), n_short, nodes);
        np_linspace(dt_short * n_short, T, N - n_short + 1, nodes + n_short);
    }
    for (int k = 0; k < N; ++k) dt[k] = nodes[k + 1] - nodes[k];
    return SDFNMPC_OK;
}

// ------------------------------------------------------------------------------------------------
// in-loop VAE encoder: .vaew blob -> device weights + activation workspace
struct VaeLayer {
    const float* w = nullptr;
    const float* b = nullptr;
    const unsigned short* wpl = nullptr;  // convolutions: w split into bf16 planes (VaeConvArgs::wpl)
    int cin = 0, cout = 0, ks = 0, stride = 0;
};

struct sdfnmpc_vae {
    int device = 0;
    int L = 0, H = 0, W = 0;
    int Hc = 0, Wc = 0, Hp = 0, Wp = 0;
    int bh[4] = {0}, bw[4] = {0};  // block output maps
    void* dmem = nullptr;
    VaeLayer stem, conv[11], head;  // conv: b0a b0s b0b b1a b1s b1b b2a b2s b2b b3a b3b
    const unsigned short* stem_wpl = nullptr;  // the stem weights split into bf16 planes (VaeStemArgs::wpl)
    const float* zero16 = nullptr;              // 16 zero floats (VaeConvArgs::zero: a tap outside the map)
    DevBuf ws;
    int ws_B = 0;
};

static const int kVaeBlockIn[4] = {64, 128, 256, 512};
static const int kVaeBlockStride[4] = {2, 2, 2, 1};

extern "C" int sdfnmpc_vae_load(sdfnmpc_ctx* ctx, const void* blob, size_t bytes, sdfnmpc_vae** out) {
    if (!ctx || !blob || !out) return fail(SDFNMPC_E_ARG, "NULL argument to sdfnmpc_vae_load");
    *out = nullptr;
    struct Hdr {
        char magic[8];
        uint32_t version, nb_chan, L, H, W, n_convs, n_floats, reserved;
    } h;
    if (bytes < sizeof(Hdr)) return fail(SDFNMPC_E_FORMAT, "vaew: truncated header");
    memcpy(&h, blob, sizeof(Hdr));
    if (memcmp(h.magic, "SDFNVAEW", 8) != 0 || h.version != 1) return fail(SDFNMPC_E_FORMAT, "not a version-1 .vaew blob");
    if (h.nb_chan != 1 || h.n_convs != 13 || h.L < 1 || h.L > 4096 || h.H < 8 || h.W < 8 || h.H > 8192 || h.W > 8192)
        return fail(SDFNMPC_E_UNSUPPORTED, "vaew: only the 1-channel reference encoder (13 convolutions) is built");
    if (bytes != sizeof(Hdr) + 4ull * h.n_floats) return fail(SDFNMPC_E_FORMAT, "vaew: size mismatch");
    const float* src = (const float*)((const char*)blob + sizeof(Hdr));
    auto* v = new sdfnmpc_vae();
    v->device = ctx->device;
    v->L = (int)h.L; v->H = (int)h.H; v->W = (int)h.W;
    v->Hc = (v->H - 1) / 2 + 1; v->Wc = (v->W - 1) / 2 + 1;
    v->Hp = (v->Hc - 1) / 2 + 1; v->Wp = (v->Wc - 1) / 2 + 1;
    // expected layer list (vae.py:device_layers) and host re-layout of stem / head
    struct Spec { int cin, cout, ks, stride; };
    std::vector<Spec> specs = {{1, 64, 7, 2}};
    int hh = v->Hp, ww = v->Wp;
    for (int k = 0; k < 4; ++k) {
        const int ci = kVaeBlockIn[k], s = kVaeBlockStride[k], co = ci * s;
        specs.push_back({ci, co, 3, s});
        if (s != 1) specs.push_back({ci, co, 1, s});
        specs.push_back({co, co, 3, 1});
        hh = (hh - 1) / s + 1;
        ww = (ww - 1) / s + 1;
        v->bh[k] = hh;
        v->bw[k] = ww;
    }
    specs.push_back({2048, (int)h.L, 1, 1});
    size_t need = 0;
    for (auto& s : specs) need += (size_t)s.cout * s.ks * s.ks * s.cin + s.cout;
    if (need != h.n_floats) {
        delete v;
        return fail(SDFNMPC_E_FORMAT, "vaew: parameter count does not match the reference encoder");
    }
    // + the stem weights split exactly into three bf16 planes [3][64 n][64 k] (vae_enc.hip's split3), in
    // the kernel's K order (vae_stem_slot_tap), appended after the layers (16-byte aligned), then every
    // ResBlock convolution's weights split the same way into planes of K-tile slabs (16-byte aligned each)
    auto split3 = [](float x, unsigned short* hi, unsigned short* mid, unsigned short* lo) {
        uint32_t u, hb, mb, lb;
        memcpy(&u, &x, 4);
        hb = u & 0xffff0000u;
        float hf, r1, mf, r2;
        memcpy(&hf, &hb, 4);
        r1 = x - hf;  // exact (the leading 8 significant bits removed)
        memcpy(&u, &r1, 4);
        mb = u & 0xffff0000u;
        memcpy(&mf, &mb, 4);
        r2 = r1 - mf;
        memcpy(&u, &r2, 4);
        lb = u & 0xffff0000u;
        *hi = (unsigned short)(hb >> 16);
        *mid = (unsigned short)(mb >> 16);
        *lo = (unsigned short)(lb >> 16);
    };
    const size_t wpl_off = (need + 3) & ~(size_t)3;
    size_t cpl_end = wpl_off + 3 * VAE_STEM_PLANE / 2;  // in floats
    std::vector<size_t> cpl_off(specs.size(), 0);
    for (size_t li = 1; li + 1 < specs.size(); ++li) {
        cpl_off[li] = cpl_end;
        const size_t nw = (size_t)specs[li].cout * specs[li].ks * specs[li].ks * specs[li].cin;
        cpl_end += ((3 * nw + 1) / 2 + 3) & ~(size_t)3;
    }
    const size_t zero_off = cpl_end;  // + 16 zero floats: what a convolution tap outside the map reads
    std::vector<float> dev(cpl_end + 16, 0.0f);
    size_t off = 0;
    for (size_t li = 0; li < specs.size(); ++li) {
        const Spec& s = specs[li];
        const size_t nw = (size_t)s.cout * s.ks * s.ks * s.cin;
        if (li == 0) {  // stem [64][7][7][1] -> tap-major [49][64], and the split planes
            unsigned short* wpl = (unsigned short*)&dev[wpl_off];
            for (int c = 0; c < 64; ++c)
                for (int t = 0; t < 49; ++t) dev[off + t * 64 + c] = src[off + c * 49 + t];
            for (int c = 0; c < 64; ++c)
                for (int k = 0; k < 49; ++k)
                    split3(src[off + c * 49 + vae_stem_slot_tap(k)], &wpl[0 * VAE_STEM_PLANE + c * 64 + k],
                           &wpl[1 * VAE_STEM_PLANE + c * 64 + k], &wpl[2 * VAE_STEM_PLANE + c * 64 + k]);
        } else if (li + 1 == specs.size()) {  // head [L][2048] -> [2048][L]
            for (int o = 0; o < s.cout; ++o)
                for (int f = 0; f < 2048; ++f) dev[off + (size_t)f * s.cout + o] = src[off + (size_t)o * 2048 + f];
        } else {
            memcpy(&dev[off], src + off, nw * 4);
            unsigned short* pl = (unsigned short*)&dev[cpl_off[li]];
            // K-tile slabs in vae_conv_kernel's K order (channel block, ky, kx): weight (n, ky, kx, ci) goes
            // to K-tile t = (ci / 16) KS KS + ky KS + kx, plane element ((n / 128 KT + t) 128 + n % 128) 16
            // + ci % 16 with the two 8-element halves of rows with bit 3 set swapped -- the LDS image of the
            // kernel's B tile, so its LDS-DMA reads 1 KB contiguous per wave (one slab: 4 KB per plane)
            const int KK = s.ks * s.ks, K = KK * s.cin, KT = K / 16;
            for (int n = 0; n < s.cout; ++n)
                for (int k = 0; k < K; ++k) {
                    const int tp = k / s.cin, ci = k % s.cin, t = (ci / 16) * KK + tp, c = ci % 16;
                    const int r = n % 128, h = (c / 8) ^ ((r >> 3) & 1);
                    const size_t e = (((size_t)(n / 128) * KT + t) * 128 + r) * 16 + 8 * h + c % 8;
                    split3(src[off + (size_t)n * K + k], &pl[e], &pl[nw + e], &pl[2 * nw + e]);
                }
        }
        memcpy(&dev[off + nw], src + off + nw, (size_t)s.cout * 4);
        off += nw + s.cout;
    }
    ScopedDevice sd(ctx->device);
    if (hipMalloc(&v->dmem, dev.size() * 4) != hipSuccess ||
        hipMemcpy(v->dmem, dev.data(), dev.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
        if (v->dmem) (void)hipFree(v->dmem);
        delete v;
        return fail(SDFNMPC_E_HIP, "vaew: device upload failed");
    }
    const float* d = (const float*)v->dmem;
    v->stem_wpl = (const unsigned short*)(d + wpl_off);
    v->zero16 = d + zero_off;
    off = 0;
    for (size_t li = 0; li < specs.size(); ++li) {
        const Spec& s = specs[li];
        VaeLayer L{d + off, d + off + (size_t)s.cout * s.ks * s.ks * s.cin,
                   cpl_off[li] ? (const unsigned short*)(d + cpl_off[li]) : nullptr, s.cin, s.cout, s.ks, s.stride};
        if (li == 0) v->stem = L;
        else if (li + 1 == specs.size()) v->head = L;
        else v->conv[li - 1] = L;
        off += (size_t)s.cout * s.ks * s.ks * s.cin + s.cout;
    }
    *out = v;
    return SDFNMPC_OK;
}

extern "C" void sdfnmpc_vae_free(sdfnmpc_vae* v) {
    if (!v) return;
    ScopedDevice sd(v->device);
    if (v->dmem) (void)hipFree(v->dmem);
    delete v;
}

extern "C" int sdfnmpc_vae_size_latent(const sdfnmpc_vae* v) { return v ? v->L : -1; }

extern "C" int sdfnmpc_vae_encode(sdfnmpc_ctx* ctx, sdfnmpc_vae* v, const sdfnmpc_vae_opts* o, const void* img,
                                  float* latent, double* latent64) {
    if (!ctx || !v || !o) return fail(SDFNMPC_E_ARG, "NULL argument to sdfnmpc_vae_encode");
    if (o->B < 0 || (o->B > 0 && (!img || !latent))) return fail(SDFNMPC_E_ARG, "vae_encode: bad B or NULL image / latent");
    if (o->dtype != 0 && o->dtype != 1) return fail(SDFNMPC_E_ARG, "vae_encode: dtype must be 0 (float32) or 1 (uint16)");
    if (o->in_h < 1 || o->in_w < 1 || !(o->clip > 0.f)) return fail(SDFNMPC_E_ARG, "vae_encode: bad image size or clip");
    if (ctx->device != v->device) return fail(SDFNMPC_E_ARG, "vae_encode: encoder loaded on another device");
    const int B = o->B;
    if (B == 0) return SDFNMPC_OK;
    ScopedDevice sd(ctx->device);
    // workspace: pre [B][H][W] | X | Y (block in/out ping-pong, bf16 planes) | T (conv_a, planes) | S (shortcut,
    // fp32) | F (head features).  A planes tensor of n values per image: [3][B][n] bf16, plane stride B n.
    const size_t n_pre = (size_t)v->H * v->W;
    size_t n_x = (size_t)v->Hp * v->Wp * 64, n_t = 0;
    for (int k = 0; k < 4; ++k) {
        const size_t nb = (size_t)v->bh[k] * v->bw[k] * kVaeBlockIn[k] * kVaeBlockStride[k];
        n_x = std::max(n_x, nb);
        n_t = std::max(n_t, nb);
    }
    // in floats per image: planes take 1.5 floats a value (n_x, n_t are multiples of 64: every plane 16-byte
    // aligned once X is); the preprocessed images [B][H][W] are padded to a multiple of 64 floats, so X (and every
    // plane after it, staged by 16-byte LDS-DMA) starts 256-byte aligned for any H, W, B
    const size_t pre_pad = (n_pre * B + 63) & ~(size_t)63;
    const size_t per = n_pre + 2 * (3 * n_x / 2) + 3 * n_t / 2 + n_t + 2048;
    HIPCHK(v->ws.ensure((per * B + 64) * sizeof(float)));
    float* P = (float*)v->ws.p;
    unsigned short* X = (unsigned short*)(P + pre_pad);
    unsigned short* Y = X + 3 * n_x * B;
    unsigned short* T = Y + 3 * n_x * B;
    float* S = (float*)(T + 3 * n_t * B);
    float* F = S + n_t * B;  // [B][2048] pooled head features
    const unsigned short* zero = (const unsigned short*)v->zero16;
    hipStream_t st = ctx->stream;
    VaePreArgs pa{img, o->dtype, B, o->in_h, o->in_w, v->H, v->W, o->clip, o->yz, P};
    HIPCHK(timed(ctx, "vae_pre", [&] { return launch_vae_pre(pa, st); }));
    size_t xps = (size_t)B * v->Hp * v->Wp * 64;  // the plane stride of the tensor in X
    // a map read by a stride-2 convolution is stored in parity-phase column order (vae_col)
    auto phased = [](int k) { return k < 4 && kVaeBlockStride[k] == 2 ? 1 : 0; };
    VaeStemArgs sa{P, v->stem_wpl, v->stem.b, X, xps, B, v->H, v->W, v->Hc, v->Wc, v->Hp, v->Wp, phased(0)};
    HIPCHK(timed(ctx, "vae_stem", [&] { return launch_vae_stem(sa, ctx->n_cu, st); }));
    int h = v->Hp, w = v->Wp, li = 0;
    for (int k = 0; k < 4; ++k) {
        const int s = kVaeBlockStride[k], ho = v->bh[k], wo = v->bw[k];
        const VaeLayer& ca = v->conv[li++];
        const size_t ops = (size_t)B * ho * wo * ca.cout;  // plane stride of this block's outputs
        const int in_ph = phased(k), out_ph = phased(k + 1);
        VaeConvArgs a1{X, xps, ca.w, ca.wpl, ca.b, zero, nullptr, nullptr, 0, nullptr, T, ops,
                       B, h, w, ca.cin, ho, wo, ca.cout, 1, in_ph, 0, 0};
        HIPCHK(timed(ctx, "vae_conv", [&] { return launch_vae_conv(a1, 3, s, st); }));
        const float* resid = nullptr;
        const unsigned short* resid_pl = X;  // identity shortcut: the block input, as planes
        int res_ph = in_ph;
        if (s != 1) {
            const VaeLayer& cs = v->conv[li++];
            VaeConvArgs a2{X, xps, cs.w, cs.wpl, cs.b, zero, nullptr, nullptr, 0, S, nullptr, 0,
                           B, h, w, cs.cin, ho, wo, cs.cout, 0, in_ph, out_ph, 0};
            HIPCHK(timed(ctx, "vae_conv", [&] { return launch_vae_conv(a2, 1, s, st); }));
            resid = S;
            resid_pl = nullptr;
            res_ph = out_ph;
        }
        const VaeLayer& cb = v->conv[li++];
        VaeConvArgs a3{T, ops, cb.w, cb.wpl, cb.b, zero, resid, resid_pl, xps, nullptr, Y, ops,
                       B, ho, wo, cb.cin, ho, wo, cb.cout, 1, 0, out_ph, res_ph};
        HIPCHK(timed(ctx, "vae_conv", [&] { return launch_vae_conv(a3, 3, 1, st); }));
        std::swap(X, Y);
        xps = ops;
        h = ho;
        w = wo;
    }
    VaeHeadArgs ha{X, xps, F, v->head.w, v->head.b, latent, latent64, B, h, w, v->L};
    HIPCHK(timed(ctx, "vae_head", [&] { return launch_vae_head(ha, st); }));
    return SDFNMPC_OK;
}
