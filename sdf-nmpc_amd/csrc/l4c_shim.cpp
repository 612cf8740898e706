// libsdf_l4c.so: the CasADi external-function ABI (include/sdf_l4c.h) over the HIP SDF path.
//
// Replaces the L4CasADi-generated libtorch library (gen_model.py:38-39).  acados calls sdf_l4c then
// jac_sdf_l4c on the same input for every shooting node, so the forward call
// computes value AND full 1 x (3 + L) gradient in one device launch and the Jacobian/adjoint calls are
// served from a per-thread cache keyed on the exact input bits.  The input width is the loaded network's:
// 3 + size_latent (gen_model.py:60 feeds vertcat(Co_p_B, latent); neural_df.py:16), 131 for the deployed
// net, any latent up to 1024 otherwise.
#include <dlfcn.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/sdf_l4c.h"
#include "../../include/sdfnmpc.h"

namespace {

std::mutex g_mu;
sdfnmpc_ctx* g_ctx = nullptr;
sdfnmpc_net* g_net = nullptr;
std::atomic<int> g_D{0};              // 3 + size_latent of the loaded network (0: not loaded)
std::string g_err;                    // guarded by g_mu
std::atomic<unsigned long long> g_gen{1};  // bumped by every sdf_l4c_configure: invalidates all caches

// per-thread cache of the last input (acados calls sdf_l4c then jac_sdf_l4c on the same input); an
// entry is valid only for the configuration generation it was computed under
thread_local std::vector<double> t_in, t_grad;
thread_local double t_df = 0.0;
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

std::string weights_path(const char* path) {
    std::string wpath = path ? path : "";
    if (wpath.empty()) {
        const char* env = getenv("SDFNMPC_WEIGHTS");
        wpath = env && *env ? env : lib_dir() + "/sdf_l4c.sdfw";
    }
    return wpath;
}

// 3 + size_latent from the .sdfw header (magic, version, nb_states, L, ...), without touching a device:
// CasADi asks for the sparsity patterns when it builds the OCP, possibly on a host without the GPU
int header_width(const std::string& wpath) {
    FILE* f = fopen(wpath.c_str(), "rb");
    if (!f) return 0;
    unsigned char h[20];
    const size_t n = fread(h, 1, sizeof h, f);
    fclose(f);
    uint32_t ver = 0, L = 0;
    if (n != sizeof h || memcmp(h, "SDFNMPCW", 8) != 0) return 0;
    memcpy(&ver, h + 8, 4);
    memcpy(&L, h + 16, 4);
    return (ver == 1 || ver == 2) && L <= 4096 ? 3 + (int)L : 0;
}

int init_locked(const char* path, int device) {
    if (g_net) return 0;
    const std::string wpath = weights_path(path);
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
    g_D.store(3 + sdfnmpc_net_size_latent(g_net));
    return 0;
}

std::string g_cfg_path;  // the weights path of the last sdf_l4c_configure (guarded by g_mu)

constexpr int DEPLOYED_WIDTH = 3 + 128;  // the deployed network's input (default.yaml nn.size_latent)
std::atomic<int> g_handed{0};            // the width of the last sparsity pattern handed to CasADi

// the input width: the loaded network's, else the header of the file the first call will load
// (CasADi asks for the sparsity before any call, possibly on a host without the GPU), else the
// deployed network's
int width() {
    const int d = g_D.load();
    if (d) return d;
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_D.load()) return g_D.load();
    const int w = header_width(weights_path(g_cfg_path.empty() ? nullptr : g_cfg_path.c_str()));
    return w ? w : DEPLOYED_WIDTH;
}

// value + gradient for one input, cached per thread
int eval(const double* in) {
    if (!in) return 1;
    const int D = width();
    if (!D) return 1;
    if (t_gen == g_gen.load() && (int)t_in.size() == D && memcmp(in, t_in.data(), D * sizeof(double)) == 0) return 0;
    std::lock_guard<std::mutex> lk(g_mu);
    if (init_locked(nullptr, -1)) return 1;
    const unsigned long long gen = g_gen.load();
    const int d = g_D.load();  // the network may have changed since width() (sdf_l4c_configure)
    const int hw = g_handed.load();
    if (hw && hw != d) {  // CasADi sized its buffers from a pattern of another width
        g_err = "sdf_l4c: the loaded network takes " + std::to_string(d) + " inputs, the sparsity pattern handed out " +
                std::to_string(hw);
        t_gen = 0;
        return 1;
    }
    t_grad.resize(d);
    if (sdfnmpc_sdf_eval_host(g_ctx, g_net, 1, in, &t_df, t_grad.data()) != SDFNMPC_OK) {
        g_err = std::string("sdf_l4c: ") + sdfnmpc_last_error();
        t_gen = 0;
        return 1;
    }
    t_in.assign(in, in + d);
    t_gen = gen;
    return 0;
}

// CasADi compressed-column sparsity patterns of width D: dense D x 1 input, 1 x 1 output, dense 1 x D
// Jacobian.  Kept per width for the life of the library (CasADi keeps the pointers it is handed).
struct Sp {
    std::vector<long long> in, scalar, row;
    explicit Sp(int D) : in(4 + D), scalar(5), row(2 + D + 1 + D) {
        in[0] = D; in[1] = 1; in[2] = 0; in[3] = D;
        for (int i = 0; i < D; ++i) in[4 + i] = i;
        scalar[0] = 1; scalar[1] = 1; scalar[2] = 0; scalar[3] = 1; scalar[4] = 0;
        row[0] = 1; row[1] = D;
        for (int j = 0; j <= D; ++j) row[2 + j] = j;
        for (int j = 0; j < D; ++j) row[2 + D + 1 + j] = 0;
    }
};
const Sp* sp() {
    static std::mutex mu;
    static std::vector<Sp*> all;  // never freed: pointers handed out stay valid
    const int D = width();
    if (!D) return nullptr;
    g_handed.store(D);
    std::lock_guard<std::mutex> lk(mu);
    for (Sp* s : all)
        if ((int)s->in[0] == D) return s;
    all.push_back(new Sp(D));
    return all.back();
}
const long long* sp_in() { const Sp* s = sp(); return s ? s->in.data() : nullptr; }
const long long* sp_scalar() { const Sp* s = sp(); return s ? s->scalar.data() : nullptr; }
const long long* sp_row() { const Sp* s = sp(); return s ? s->row.data() : nullptr; }

}  // namespace

extern "C" {

int sdf_l4c_configure(const char* weights_path, int device) {
    std::lock_guard<std::mutex> lk(g_mu);
    // CasADi keeps the sparsity patterns it was handed and sizes its argument / result buffers from them:
    // once a pattern of width hw is out, a network of another width would read past the caller's input and
    // write past its Jacobian buffer.  Refused before anything is freed; the loaded network stays.
    const int hw = g_handed.load();
    if (hw) {
        const int w = header_width(::weights_path(weights_path));
        if (w != hw) {
            g_err = "sdf_l4c_configure: a sparsity pattern of width " + std::to_string(hw) +
                    " was handed out; the network takes " + (w ? std::to_string(w) : std::string("(unreadable)")) +
                    " inputs (one width per process)";
            return 1;
        }
    }
    g_gen++;  // every thread's cached value / gradient belongs to the previous network
    if (g_net) {
        sdfnmpc_net_free(g_net);
        g_net = nullptr;
    }
    if (g_ctx) {
        sdfnmpc_ctx_destroy(g_ctx);
        g_ctx = nullptr;
    }
    g_D.store(0);
    g_cfg_path = weights_path ? weights_path : "";
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
const long long* sdf_l4c_sparsity_in(long long i) { return i == 0 ? sp_in() : nullptr; }
const long long* sdf_l4c_sparsity_out(long long i) { return i == 0 ? sp_scalar() : nullptr; }
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
    if (res[0]) memcpy(res[0], t_grad.data(), t_grad.size() * sizeof(double));
    return 0;
}
long long jac_sdf_l4c_n_in(void) { return 2; }
long long jac_sdf_l4c_n_out(void) { return 1; }
const long long* jac_sdf_l4c_sparsity_in(long long i) { return i == 0 ? sp_in() : (i == 1 ? sp_scalar() : nullptr); }
const long long* jac_sdf_l4c_sparsity_out(long long i) { return i == 0 ? sp_row() : nullptr; }
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
        for (size_t i = 0; i < t_grad.size(); ++i) res[0][i] = seed * t_grad[i];
    return 0;
}
long long adj1_sdf_l4c_n_in(void) { return 3; }
long long adj1_sdf_l4c_n_out(void) { return 1; }
const long long* adj1_sdf_l4c_sparsity_in(long long i) {
    return i == 0 ? sp_in() : ((i == 1 || i == 2) ? sp_scalar() : nullptr);
}
const long long* adj1_sdf_l4c_sparsity_out(long long i) { return i == 0 ? sp_in() : nullptr; }
int adj1_sdf_l4c_work(long long* a, long long* r, long long* iw, long long* w) {
    if (a) *a = 3;
    if (r) *r = 1;
    if (iw) *iw = 0;
    if (w) *w = 0;
    return 0;
}

}  // extern "C"
