// sdfnmpc_solver: the device-resident SQP-RTI solver object of include/sdfnmpc.h.
//
// It owns everything one batched control step touches -- iterate, parameters, references, the
// preparation-phase outputs, QP results -- on one context (device + stream), so a controller drives
// it with host arrays and no tensor framework: the counterpart of the AcadosOcpSolver object that
// sdf_nmpc/ocp.py:127 builds (solver.set / cost_set / get / solve_for_x0 / reset), batched over B
// instances.  The compute is the lower-level entry points (sdfnmpc_rti_prepare, sdfnmpc_qp_feedback,
// sdfnmpc_rti_apply); this file adds buffer ownership, masked row uploads through a pinned staging
// arena, and the asynchronous step / wait split that lets one host thread keep several devices busy.
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <vector>

#include "../../include/sdfnmpc.h"

extern "C" int sdfnmpc_solver_fail_(int code, const char* msg);  // engine.cpp: sets sdfnmpc_last_error

namespace {

#define SCHK(expr)                                                                                       \
    do {                                                                                                 \
        hipError_t e_ = (expr);                                                                          \
        if (e_ != hipSuccess)                                                                            \
            return sdfnmpc_solver_fail_(SDFNMPC_E_HIP, (std::string(#expr) + ": " + hipGetErrorString(e_)).c_str()); \
    } while (0)

// rows r of a [rows][width] field receive staged[r'][0..ncol) at columns col0.. (r = idx[r'])
__global__ __launch_bounds__(256) void scatter_rows_kernel(double* dst, int width, int col0, int ncol,
                                                           const double* staged, const int* idx, int n_rows) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)n_rows * ncol) return;
    const int r = (int)(i / ncol), c = (int)(i - (long long)r * ncol);
    dst[(long long)idx[r] * width + col0 + c] = staged[i];
}

// x_{i-k} = x_i, u_{i-k} = u_i for i = k..N-1 (ocp.py:152-156): one thread per (instance, column), nodes in
// ascending order, so the overlapping rows are read before they are overwritten
__global__ __launch_bounds__(256) void shift_kernel(int B, int N, int k, double* x, double* u) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)B * 14) return;
    const long long b = i / 14;
    const int j = (int)(i - b * 14);
    if (j < 10) {
        double* xb = x + b * (N + 1) * 10 + j;
        for (int n = k; n < N; ++n) xb[(n - k) * 10] = xb[n * 10];
    } else {
        double* ub = u + b * N * 4 + (j - 10);
        for (int n = k; n < N; ++n) ub[(n - k) * 4] = ub[n * 4];
    }
}

// x[b][k] = x0[b] (k = 0..N), u[b][k] = u_init (k < N)
__global__ __launch_bounds__(256) void init_iterate_kernel(int B, int N, double* x, double* u, const double* x0,
                                                           double u0, double u1, double u2, double u3) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long nx = (long long)B * (N + 1) * 10, nu = (long long)B * N * 4;
    if (i < nx) {
        const long long b = i / ((N + 1) * 10), e = i % 10;
        x[i] = x0[b * 10 + e];
    }
    if (i < nu) {
        const int e = (int)(i & 3);
        u[i] = e == 0 ? u0 : e == 1 ? u1 : e == 2 ? u2 : u3;
    }
}

struct Field {
    const char* name;
    void* dev;
    int nodes, width, elem;  // [B][nodes][width] of elem-byte values
};

}  // namespace

struct sdfnmpc_solver {
    sdfnmpc_ctx* ctx = nullptr;
    const sdfnmpc_net* net = nullptr;
    int device = 0;
    hipStream_t stream = nullptr;
    int B = 0, N = 0, np = 0, ny = 0, nyN = 4, latent_mode = 0;
    bool no_sdf = false;  // no constraint row or cost reads the network
    sdfnmpc_quad_model model{};
    sdfnmpc_qp_opts qp{};
    std::vector<void*> allocs;
    double *x = nullptr, *u = nullptr, *p = nullptr, *x0 = nullptr, *yref = nullptr, *W = nullptr, *yNref = nullptr,
           *WN = nullptr, *dt = nullptr, *xn = nullptr, *AB = nullptr, *y = nullptr, *Jy = nullptr, *yN = nullptr,
           *JyN = nullptr, *h = nullptr, *Jh = nullptr, *dx = nullptr, *du = nullptr, *res = nullptr, *u0 = nullptr,
           *slack = nullptr, *hE = nullptr, *JhE = nullptr;
    int *status = nullptr, *iters = nullptr;
    // pinned host memory: step outputs and the upload staging arena (reset after every wait)
    double* h_u0 = nullptr;
    int *h_status = nullptr, *h_iters = nullptr;
    char* arena = nullptr;   // pinned host staging
    char* d_arena = nullptr; // its device twin (same offsets): staged rows land here before the scatter
    size_t arena_bytes = 0, arena_used = 0;
    bool pending = false;
    std::vector<Field> fields;

    ~sdfnmpc_solver() {
        int prev = -1;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(device);
        (void)hipStreamSynchronize(stream);
        for (void* a : allocs) (void)hipFree(a);
        if (d_arena) (void)hipFree(d_arena);
        if (h_u0) (void)hipHostFree(h_u0);  // [u0 | status | iters] in one pinned block
        if (arena) (void)hipHostFree(arena);
        if (prev >= 0) (void)hipSetDevice(prev);
    }

    template <typename T>
    hipError_t alloc(T** out, size_t n) {
        void* q = nullptr;
        hipError_t e = hipMalloc(&q, n * sizeof(T) + 16);
        if (e != hipSuccess) return e;
        allocs.push_back(q);
        e = hipMemsetAsync(q, 0, n * sizeof(T), stream);
        *out = (T*)q;
        return e;
    }
    const Field* field(const char* name) const {
        for (const Field& f : fields)
            if (!strcmp(f.name, name)) return &f;
        return nullptr;
    }
    // n bytes of pinned staging (host pointer *out, device twin *dout), 16-byte aligned; when full the
    // stream is drained (every copy out of the arena has completed) and the arena reused or grown
    hipError_t stage(size_t n, char** out, char** dout = nullptr) {
        n = (n + 15) & ~(size_t)15;
        if (arena_used + n > arena_bytes) {
            hipError_t e = hipStreamSynchronize(stream);
            if (e != hipSuccess) return e;
            arena_used = 0;
            if (n > arena_bytes) {
                if (arena) (void)hipHostFree(arena);
                if (d_arena) (void)hipFree(d_arena);
                arena = d_arena = nullptr;
                arena_bytes = 0;
                const size_t want = n > (1u << 20) ? 2 * n : (1u << 20);
                e = hipHostMalloc((void**)&arena, want, hipHostMallocDefault);
                if (e == hipSuccess) e = hipMalloc((void**)&d_arena, want);
                if (e != hipSuccess) return e;
                arena_bytes = want;
            }
        }
        *out = arena + arena_used;
        if (dout) *dout = d_arena + arena_used;
        arena_used += n;
        return hipSuccess;
    }
};

struct SolverDevice {
    int prev = -1;
    explicit SolverDevice(int d) {
        (void)hipGetDevice(&prev);
        if (prev != d) (void)hipSetDevice(d);
    }
    ~SolverDevice() {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
    }
};

extern "C" int sdfnmpc_solver_create(sdfnmpc_ctx* ctx, const sdfnmpc_net* net, const sdfnmpc_solver_opts* o,
                                     sdfnmpc_solver** out) {
    if (!ctx || !o || !out) return sdfnmpc_solver_fail_(SDFNMPC_E_ARG, "NULL argument to sdfnmpc_solver_create");
    *out = nullptr;
    if (o->B < 1 || o->N < 1 || o->np < 17 || (o->ny != 11 && o->ny != 12) || !o->dt ||
        (o->latent_mode != 0 && o->latent_mode != 1) || o->qp.ny != o->ny)
        return sdfnmpc_solver_fail_(SDFNMPC_E_ARG, "solver opts: B, N >= 1, np >= 17, ny in {11, 12} == qp.ny, dt required");
    if (o->qp.nyN != 4 && o->qp.nyN != 5)
        return sdfnmpc_solver_fail_(SDFNMPC_E_ARG, "solver opts: qp.nyN must be 4 or 5");
    bool need_sdf = o->ny == 12;  // the constraint set or the cost reads the network
    for (int j = 0; j < o->qp.nh && j < 3; ++j) need_sdf = need_sdf || o->qp.h_col[j] == 2;
    for (int j = 0; j < o->qp.nhN && j < SDFNMPC_NHN_MAX; ++j) need_sdf = need_sdf || o->qp.hN_col[j] == 2;
    if (need_sdf && !net)
        return sdfnmpc_solver_fail_(SDFNMPC_E_ARG, "solver: the constraint set / cost reads the SDF but the network is NULL");
    if (net && o->np < 17 + sdfnmpc_net_size_latent(net))  // the stage parameters end with the network's latent
        return sdfnmpc_solver_fail_(SDFNMPC_E_ARG, ("solver opts: np = " + std::to_string(o->np) + " < 17 + latent size " +
                                                    std::to_string(sdfnmpc_net_size_latent(net)) + " of this network").c_str());
    auto* s = new sdfnmpc_solver();
    s->ctx = ctx;
    s->net = net;
    s->device = sdfnmpc_ctx_device(ctx);
    s->stream = (hipStream_t)sdfnmpc_ctx_stream(ctx);
    s->B = o->B; s->N = o->N; s->np = o->np; s->ny = o->ny; s->latent_mode = o->latent_mode;
    s->nyN = o->qp.nyN;
    s->no_sdf = !need_sdf;
    s->model = o->model;
    s->qp = o->qp;
    SolverDevice sd(s->device);
    const size_t B = o->B, N = o->N, N1 = N + 1;
    hipError_t e = hipSuccess;
    auto A = [&](auto** p, size_t n) { if (e == hipSuccess) e = s->alloc(p, n); };
    A(&s->x, B * N1 * 10); A(&s->u, B * N * 4); A(&s->p, B * N1 * o->np); A(&s->x0, B * 10);
    const size_t nyN = s->nyN;
    A(&s->yref, B * N * o->ny); A(&s->W, B * N * o->ny); A(&s->yNref, B * nyN); A(&s->WN, B * nyN); A(&s->dt, N);
    A(&s->xn, B * N * 10); A(&s->AB, B * N * 140); A(&s->y, B * N * 11); A(&s->Jy, B * N * 154); A(&s->yN, B * nyN);
    A(&s->JyN, B * 10 * nyN); A(&s->h, B * N1 * 3); A(&s->Jh, B * N1 * 30); A(&s->dx, B * N1 * 10); A(&s->du, B * N * 4);
    A(&s->res, B * 2); A(&s->slack, B * N1 * 6); A(&s->hE, B * 6); A(&s->JhE, B * 60);
    // [u0 (B x 4 doubles) | status (B ints) | iters (B ints)] contiguous on both sides: one copy back per step
    A(&s->u0, B * 5);
    if (e == hipSuccess) {
        s->status = (int*)(s->u0 + B * 4);
        s->iters = s->status + B;
        e = hipHostMalloc((void**)&s->h_u0, B * 5 * sizeof(double), hipHostMallocDefault);
    }
    if (e == hipSuccess) {
        s->h_status = (int*)(s->h_u0 + B * 4);
        s->h_iters = s->h_status + B;
    }
    if (e == hipSuccess) e = hipMemcpyAsync(s->dt, o->dt, N * sizeof(double), hipMemcpyHostToDevice, s->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    if (e != hipSuccess) {
        delete s;
        return sdfnmpc_solver_fail_(SDFNMPC_E_HIP, (std::string("solver buffers: ") + hipGetErrorString(e)).c_str());
    }
    const int n = (int)N, n1 = (int)N1, d = 8, w = (int)nyN;
    s->fields = {{"x", s->x, n1, 10, d},       {"u", s->u, n, 4, d},          {"p", s->p, n1, o->np, d},
                 {"x0", s->x0, 1, 10, d},      {"yref", s->yref, n, o->ny, d}, {"W", s->W, n, o->ny, d},
                 {"yNref", s->yNref, 1, w, d}, {"WN", s->WN, 1, w, d},         {"u0", s->u0, 1, 4, d},
                 {"dx", s->dx, n1, 10, d},     {"du", s->du, n, 4, d},         {"xn", s->xn, n, 10, d},
                 {"AB", s->AB, n, 140, d},     {"y", s->y, n, 11, d},          {"Jy", s->Jy, n, 154, d},
                 {"yN", s->yN, 1, w, d},       {"JyN", s->JyN, 1, 10 * w, d},  {"h", s->h, n1, 3, d},
                 {"Jh", s->Jh, n1, 30, d},     {"hE", s->hE, 1, 6, d},         {"JhE", s->JhE, 1, 60, d},
                 {"res", s->res, 1, 2, d},     {"slack", s->slack, n1, 6, d},  {"status", s->status, 1, 1, 4},
                 {"iters", s->iters, 1, 1, 4}};
    *out = s;
    return SDFNMPC_OK;
}

extern "C" void sdfnmpc_solver_destroy(sdfnmpc_solver* s) { delete s; }

extern "C" int sdfnmpc_solver_field(sdfnmpc_solver* s, const char* name, void** dev, int* nodes, int* width) {
    if (!s || !name) return sdfnmpc_solver_fail_(SDFNMPC_E_ARG, "NULL argument to sdfnmpc_solver_field");
    const Field* f = s->field(name);
    if (!f) return sdfnmpc_solver_fail_(SDFNMPC_E_ARG, (std::string("no solver field ") + name).c_str());
    if (dev) *dev = f->dev;
    if (nodes) *nodes = f->nodes;
    if (width) *width = f->width;
    return SDFNMPC_OK;
}

extern "C" int sdfnmpc_solver_upload(sdfnmpc_solver* s, const char* name, int col0, int ncol, const unsigned char* mask,
                                     const double* host) {
    if (!s || !name || !host) return sdfnmpc_solver_fail_(SDFNMPC_E_ARG, "NULL argument to sdfnmpc_solver_upload");
    const Field* f = s->field(name);
    if (!f || f->elem != 8) return sdfnmpc_solver_fail_(SDFNMPC_E_ARG, (std::string("no fp64 solver field ") + name).c_str());
    if (col0 < 0 || ncol < 1 || col0 + ncol > f->width) return sdfnmpc_solver_fail_(SDFNMPC_E_ARG, "upload columns out of range");
    SolverDevice sd(s->device);
    const int rows = s->B * f->nodes;
    if (!mask && col0 == 0 && ncol == f->width) {  // the whole field: one staged copy
        char* st = nullptr;
        const size_t bytes = (size_t)rows * f->width * 8;
        SCHK(s->stage(bytes, &st));
        memcpy(st, host, bytes);
        SCHK(hipMemcpyAsync(f->dev, st, bytes, hipMemcpyHostToDevice, s->stream));
        return SDFNMPC_OK;
    }
    int n_rows = 0;
    for (int r = 0; r < rows; ++r) n_rows += (!mask || mask[r]) ? 1 : 0;
    if (n_rows == 0) return SDFNMPC_OK;
    // values and row indices in ONE reservation: a second stage() call could drain and reset the arena
    // and hand out a block overlapping the first
    char *vals = nullptr, *dvals = nullptr;
    const size_t vbytes = ((size_t)n_rows * ncol * 8 + 15) & ~(size_t)15;
    SCHK(s->stage(vbytes + (size_t)n_rows * 4, &vals, &dvals));
    char *idx = vals + vbytes, *didx = dvals + vbytes;
    double* v = (double*)vals;
    int* ix = (int*)idx;
    for (int r = 0, q = 0; r < rows; ++r)
        if (!mask || mask[r]) {
            memcpy(v + (size_t)q * ncol, host + (size_t)r * f->width + col0, (size_t)ncol * 8);
            ix[q++] = r;
        }
    SCHK(hipMemcpyAsync(dvals, vals, (size_t)n_rows * ncol * 8, hipMemcpyHostToDevice, s->stream));
    SCHK(hipMemcpyAsync(didx, idx, (size_t)n_rows * 4, hipMemcpyHostToDevice, s->stream));
    const long long n = (long long)n_rows * ncol;
    hipLaunchKernelGGL(scatter_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s->stream, (double*)f->dev,
                       f->width, col0, ncol, (const double*)dvals, (const int*)didx, n_rows);
    SCHK(hipGetLastError());
    return SDFNMPC_OK;
}

extern "C" int sdfnmpc_solver_download(sdfnmpc_solver* s, const char* name, void* host) {
    if (!s || !name || !host) return sdfnmpc_solver_fail_(SDFNMPC_E_ARG, "NULL argument to sdfnmpc_solver_download");
    const Field* f = s->field(name);
    if (!f) return sdfnmpc_solver_fail_(SDFNMPC_E_ARG, (std::string("no solver field ") + name).c_str());
    SolverDevice sd(s->device);
    SCHK(hipMemcpyAsync(host, f->dev, (size_t)s->B * f->nodes * f->width * f->elem, hipMemcpyDeviceToHost, s->stream));
    SCHK(hipStreamSynchronize(s->stream));
    return SDFNMPC_OK;
}

extern "C" int sdfnmpc_solver_init(sdfnmpc_solver* s, const double* x0, const double* u_init) {
    if (!s || !x0 || !u_init) return sdfnmpc_solver_fail_(SDFNMPC_E_ARG, "NULL argument to sdfnmpc_solver_init");
    SolverDevice sd(s->device);
    int rc = sdfnmpc_solver_upload(s, "x0", 0, 10, nullptr, x0);
    if (rc) return rc;
    const long long n = (long long)s->B * (s->N + 1) * 10;
    hipLaunchKernelGGL(init_iterate_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s->stream, s->B, s->N, s->x,
                       s->u, (const double*)s->x0, u_init[0], u_init[1], u_init[2], u_init[3]);
    SCHK(hipGetLastError());
    SCHK(hipMemsetAsync(s->dx, 0, (size_t)s->B * (s->N + 1) * 10 * 8, s->stream));
    SCHK(hipMemsetAsync(s->du, 0, (size_t)s->B * s->N * 4 * 8, s->stream));
    return SDFNMPC_OK;
}

extern "C" int sdfnmpc_solver_shift(sdfnmpc_solver* s, int k) {
    if (!s) return sdfnmpc_solver_fail_(SDFNMPC_E_ARG, "NULL solver");
    if (k <= 0 || k >= s->N) return SDFNMPC_OK;  // ocp.py:153: k > 0 shifts nodes k..N-1 down by k
    SolverDevice sd(s->device);
    // one launch (it was four strided copies through a scratch buffer: launch latency on the C1 path)
    const long long n = (long long)s->B * 14;
    hipLaunchKernelGGL(shift_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s->stream, s->B, s->N, k, s->x,
                       s->u);
    SCHK(hipGetLastError());
    return SDFNMPC_OK;
}

extern "C" int sdfnmpc_solver_step(sdfnmpc_solver* s) {
    if (!s) return sdfnmpc_solver_fail_(SDFNMPC_E_ARG, "NULL solver");
    SolverDevice sd(s->device);
    const size_t n1 = s->N + 1;
    // x_0 of the iterate = the measured state (Ocp.solve: solver.set(0, 'x', x0), ocp.py:161)
    SCHK(hipMemcpy2DAsync(s->x, n1 * 80, s->x0, 80, 80, s->B, hipMemcpyDeviceToDevice, s->stream));
    sdfnmpc_lin_args la{};
    la.B = s->B; la.N = s->N; la.np = s->np; la.latent_mode = s->latent_mode;
    la.x = s->x; la.u = s->u; la.p = s->p; la.dt = s->dt;
    la.xn = s->xn; la.AB = s->AB; la.y = s->y; la.Jy = s->Jy; la.yN = s->yN; la.JyN = s->JyN; la.h = s->h; la.Jh = s->Jh;
    la.nyN = s->nyN; la.no_sdf = s->no_sdf ? 1 : 0; la.hE = s->hE; la.JhE = s->JhE;
    sdfnmpc_qp_args qa{};
    qa.B = s->B; qa.N = s->N;
    qa.xn = s->xn; qa.AB = s->AB; qa.y = s->y; qa.Jy = s->Jy; qa.yN = s->yN; qa.JyN = s->JyN; qa.h = s->h; qa.Jh = s->Jh;
    qa.hE = s->hE; qa.JhE = s->JhE;
    qa.x = s->x; qa.u = s->u; qa.x0 = s->x0; qa.yref = s->yref; qa.W = s->W; qa.yNref = s->yNref; qa.WN = s->WN;
    qa.dt = s->dt; qa.dx = s->dx; qa.du = s->du; qa.slack = s->slack; qa.status = s->status; qa.iters = s->iters;
    qa.res = s->res;
    int rc = sdfnmpc_rti_prepare(s->ctx, s->net, &s->model, &la, &s->qp, &qa);  // preparation (+ stage records)
    if (rc) return rc;
    rc = sdfnmpc_qp_feedback(s->ctx, &s->qp, &qa);                             // feedback
    if (rc) return rc;
    rc = sdfnmpc_rti_apply(s->ctx, s->B, s->N, s->x, s->u, s->dx, s->du, s->u0, s->status);
    if (rc) return rc;
    SCHK(hipMemcpyAsync(s->h_u0, s->u0, (size_t)s->B * 40, hipMemcpyDeviceToHost, s->stream));  // u0, status, iters
    s->pending = true;
    return SDFNMPC_OK;
}

extern "C" int sdfnmpc_solver_wait(sdfnmpc_solver* s, double* u0, int* status, int* iters) {
    if (!s) return sdfnmpc_solver_fail_(SDFNMPC_E_ARG, "NULL solver");
    SolverDevice sd(s->device);
    SCHK(hipStreamSynchronize(s->stream));
    s->arena_used = 0;  // every staged upload has landed
    if (!s->pending && (u0 || status || iters))
        return sdfnmpc_solver_fail_(SDFNMPC_E_ARG, "sdfnmpc_solver_wait: no step was enqueued");
    s->pending = false;
    if (u0) memcpy(u0, s->h_u0, (size_t)s->B * 32);
    if (status) memcpy(status, s->h_status, (size_t)s->B * 4);
    if (iters) memcpy(iters, s->h_iters, (size_t)s->B * 4);
    return SDFNMPC_OK;
}
