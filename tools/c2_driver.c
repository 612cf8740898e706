/* Config C2 as acados drives it, from C: the CasADi external functions of libsdf_l4c.so called per
 * shooting node -- sdf_l4c, then jac_sdf_l4c on the same input (gen_model.py:39,60; acados evaluates the
 * nonlinear constraint h and its Jacobian at every node of an RTI) -- timed with clock_gettime, no
 * interpreter in the loop.  Measurement tool for bench.py (the ctypes figure beside it includes Python's
 * per-call overhead).  Build: gcc -O2 -o tools/_c2_driver tools/c2_driver.c -ldl
 * Usage: _c2_driver LIB WEIGHTS DEVICE NODES RTIS  -> one JSON line */
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

typedef int (*cfun)(const double**, double**, long long*, double*, int);
typedef int (*cfg_fn)(const char*, int);

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}
static int cmp(const void* a, const void* b) {
    const double x = *(const double*)a, y = *(const double*)b;
    return x < y ? -1 : x > y;
}

int main(int argc, char** argv) {
    if (argc != 6) {
        fprintf(stderr, "usage: %s LIB WEIGHTS DEVICE NODES RTIS\n", argv[0]);
        return 2;
    }
    const int dev = atoi(argv[3]), nodes = atoi(argv[4]), rtis = atoi(argv[5]);
    void* h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        fprintf(stderr, "dlopen: %s\n", dlerror());
        return 1;
    }
    cfg_fn configure = (cfg_fn)dlsym(h, "sdf_l4c_configure");
    cfun f = (cfun)dlsym(h, "sdf_l4c"), jf = (cfun)dlsym(h, "jac_sdf_l4c");
    if (!configure || !f || !jf || configure(argv[2], dev) != 0) {
        fprintf(stderr, "sdf_l4c symbols / configure failed\n");
        return 1;
    }
    enum { D = 131 };
    double* in = malloc(sizeof(double) * (size_t)nodes * D);
    double* out = malloc(sizeof(double) * (size_t)nodes);
    double* jac = malloc(sizeof(double) * (size_t)nodes * D);
    double* t = malloc(sizeof(double) * (size_t)rtis);
    unsigned s = 12345u;
    for (int k = 0; k < nodes; ++k)
        for (int i = 0; i < D; ++i) {
            s = s * 1664525u + 1013904223u;
            const double r = (double)(s >> 8) / (double)(1u << 24) * 2.0 - 1.0;
            in[k * D + i] = i < 3 ? 2.0 * r : (k == 0 ? r : in[i]);  /* one latent for every node */
        }
    for (int rep = -3; rep < rtis; ++rep) {
        const double t0 = now();
        for (int k = 0; k < nodes; ++k) {
            const double* a1[1] = {in + k * D};
            double* r1[1] = {out + k};
            const double* a2[2] = {in + k * D, out + k};
            double* r2[1] = {jac + k * D};
            if (f(a1, r1, NULL, NULL, 0) || jf(a2, r2, NULL, NULL, 0)) {
                fprintf(stderr, "sdf_l4c call failed\n");
                return 1;
            }
        }
        if (rep >= 0) t[rep] = now() - t0;
    }
    qsort(t, (size_t)rtis, sizeof(double), cmp);
    printf("{\"us_per_node\": %.3f, \"ms_per_rti\": %.4f, \"nodes_per_rti\": %d, \"rtis\": %d, \"df0\": %.9g}\n",
           t[rtis / 2] / nodes * 1e6, t[rtis / 2] * 1e3, nodes, rtis, out[0]);
    return 0;
}
