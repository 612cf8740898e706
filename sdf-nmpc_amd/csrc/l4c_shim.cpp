// libsdf_l4c.so: the CasADi external-function ABI (include/sdf_l4c.h) over the HIP SDF path.
//
// Replaces the L4CasADi-generated libtorch library (gen_model.py:38-39).  acados calls sdf_l4c then
// jac_sdf_l4c on the same input for every shooting node, so the forward call
// computes value AND full 1x131 gradient in one device launch and the Jacobian/adjoint calls are
// served from a per-thread cache keyed on the exact input bits.
#include <dlfcn.h>

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "../../include/sdf_l4c.h"
#include "../../include/sdfnmpc.h"

namespace {

constexpr int D = 131;  // 3 + latent 128

std::mutex g_mu;
sdfnmpc_ctx* g_ctx = nullptr;
sdfnmpc_net* g_net = nullptr;
std::string g_err;                    // guarded by g_mu
std::atomic<unsigned long long> g_gen{1};  // bumped by every sdf_l4c_configure: invalidates all caches

// per-thread cache of the last input (acados calls sdf_l4c then jac_sdf_l4c on the same input); an
// entry is valid only for the configuration generation it was computed under
thread_local double t_in[D];
thread_local double t_df = 0.0, t_grad[D];
thread_local unsigned long long t_gen = 0;
thread_local std::string t_err;

std::string lib_dir() {
    Dl_info info;
    if (dladdr((void*)&sdf_l4c, &info) && info.dli_fname) {
        std::string p(info.dli_fname);
        size_t s = p.rfind('/');
        return s == std::string::npos ? std::string(".") : p.substr(0, s);
    }
    return ".";
}

int init_locked(const char* path, int device) {
    if (g_net) return 0;
    std::string wpath = path ? path : "";
    if (wpath.empty()) {
        const char* env = getenv("SDFNMPC_WEIGHTS");
        wpath = env && *env ? env : lib_dir() + "/sdf_l4c.sdfw";
    }
    if (device < 0) {
        const char* env = getenv("SDFNMPC_DEVICE");
        device = env && *env ? atoi(env) : 0;
    }
    if (sdfnmpc_ctx_create(device, nullptr, &g_ctx) != SDFNMPC_OK) {
        g_err = std::string("sdf_l4c: ") + sdfnmpc_last_error();
        return -1;
    }
    if (sdfnmpc_net_load_file(g_ctx, wpath.c_str(), &g_net) != SDFNMPC_OK) {
        g_err = std::string("sdf_l4c: ") + sdfnmpc_last_error();
        sdfnmpc_ctx_destroy(g_ctx);
        g_ctx = nullptr;
        return -1;
    }
    if (sdfnmpc_net_size_latent(g_net) != D - 3) {
        g_err = "sdf_l4c: network latent size != 128";
        return -1;
    }
    return 0;
}

// value + gradient for one input, cached per thread
int eval(const double* in) {
    if (!in) return 1;
    if (t_gen == g_gen.load() && memcmp(in, t_in, sizeof t_in) == 0) return 0;
    std::lock_guard<std::mutex> lk(g_mu);
    if (init_locked(nullptr, -1)) return 1;
    const unsigned long long gen = g_gen.load();
    if (sdfnmpc_sdf_eval_host(g_ctx, g_net, 1, in, &t_df, t_grad) != SDFNMPC_OK) {
        g_err = std::string("sdf_l4c: ") + sdfnmpc_last_error();
        t_gen = 0;
        return 1;
    }
    memcpy(t_in, in, sizeof t_in);
    t_gen = gen;
    return 0;
}

// CasADi compressed-column sparsity patterns
struct Sp {
    long long in[2 + 2 + D], scalar[2 + 2 + 1], row[2 + D + 1 + D];
    Sp() {
        in[0] = D; in[1] = 1; in[2] = 0; in[3] = D;
        for (int i = 0; i < D; ++i) in[4 + i] = i;
        scalar[0] = 1; scalar[1] = 1; scalar[2] = 0; scalar[3] = 1; scalar[4] = 0;
        row[0] = 1; row[1] = D;
        for (int j = 0; j <= D; ++j) row[2 + j] = j;
        for (int j = 0; j < D; ++j) row[2 + D + 1 + j] = 0;
    }
};
const Sp& sp() {
    static Sp s;
    return s;
}

}  // namespace

extern "C" {

int sdf_l4c_configure(const char* weights_path, int device) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_gen++;  // every thread's cached value / gradient belongs to the previous network
    if (g_net) {
        sdfnmpc_net_free(g_net);
        g_net = nullptr;
    }
    if (g_ctx) {
        sdfnmpc_ctx_destroy(g_ctx);
        g_ctx = nullptr;
    }
    return init_locked(weights_path, device) ? 1 : 0;
}
const char* sdf_l4c_last_error(void) {  // a per-thread copy taken under the lock
    std::lock_guard<std::mutex> lk(g_mu);
    t_err = g_err;
    return t_err.c_str();
}

// ---- f
int sdf_l4c(const double** arg, double** res, long long*, double*, int) {
    if (!arg || !res || eval(arg[0])) return 1;
    if (res[0]) res[0][0] = t_df;
    return 0;
}
long long sdf_l4c_n_in(void) { return 1; }
long long sdf_l4c_n_out(void) { return 1; }
const long long* sdf_l4c_sparsity_in(long long i) { return i == 0 ? sp().in : nullptr; }
const long long* sdf_l4c_sparsity_out(long long i) { return i == 0 ? sp().scalar : nullptr; }
int sdf_l4c_work(long long* a, long long* r, long long* iw, long long* w) {
    if (a) *a = 1;
    if (r) *r = 1;
    if (iw) *iw = 0;
    if (w) *w = 0;
    return 0;
}
const char* sdf_l4c_name_in(long long i) { return i == 0 ? "i0" : nullptr; }
const char* sdf_l4c_name_out(long long i) { return i == 0 ? "o0" : nullptr; }
int sdf_l4c_checkout(void) { return 0; }
void sdf_l4c_release(int) {}
void sdf_l4c_incref(void) {}
void sdf_l4c_decref(void) {}

// ---- jac_f
int jac_sdf_l4c(const double** arg, double** res, long long*, double*, int) {
    if (!arg || !res || eval(arg[0])) return 1;
    if (res[0]) memcpy(res[0], t_grad, sizeof t_grad);
    return 0;
}
long long jac_sdf_l4c_n_in(void) { return 2; }
long long jac_sdf_l4c_n_out(void) { return 1; }
const long long* jac_sdf_l4c_sparsity_in(long long i) { return i == 0 ? sp().in : (i == 1 ? sp().scalar : nullptr); }
const long long* jac_sdf_l4c_sparsity_out(long long i) { return i == 0 ? sp().row : nullptr; }
int jac_sdf_l4c_work(long long* a, long long* r, long long* iw, long long* w) {
    if (a) *a = 2;
    if (r) *r = 1;
    if (iw) *iw = 0;
    if (w) *w = 0;
    return 0;
}

// ---- adj1_f
int adj1_sdf_l4c(const double** arg, double** res, long long*, double*, int) {
    if (!arg || !res || eval(arg[0])) return 1;
    const double seed = arg[2] ? arg[2][0] : 0.0;
    if (res[0])
        for (int i = 0; i < D; ++i) res[0][i] = seed * t_grad[i];
    return 0;
}
long long adj1_sdf_l4c_n_in(void) { return 3; }
long long adj1_sdf_l4c_n_out(void) { return 1; }
const long long* adj1_sdf_l4c_sparsity_in(long long i) {
    return i == 0 ? sp().in : ((i == 1 || i == 2) ? sp().scalar : nullptr);
}
const long long* adj1_sdf_l4c_sparsity_out(long long i) { return i == 0 ? sp().in : nullptr; }
int adj1_sdf_l4c_work(long long* a, long long* r, long long* iw, long long* w) {
    if (a) *a = 3;
    if (r) *r = 1;
    if (iw) *iw = 0;
    if (w) *w = 0;
    return 0;
}

}  // extern "C"
