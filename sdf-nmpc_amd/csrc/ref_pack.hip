// Batched reference / parameter packing: for B instances x (N+1) nodes,
//   RefGen.gen_ref_list_wps / gen_ref_joystick / from_x0   (sdf_nmpc/ref_gen.py:17-130)
//   -> Quad.formate_ref                                      (model/quad_rollpitchyawrate.py:62-65)
//   -> Nmpc.set_ref (q_d into p, y / W, yN / WN)             (controller.py:133-142)
//   and Nmpc.set_latent / set_sdf_flag                       (controller.py:45-54)
// in one launch that writes the OCP's device buffers, replacing 3 (N+1) host setter calls per
// instance.  One workgroup per instance; node k is computed by thread k (mod 64) from the shared path.
// Arithmetic follows the numpy order of the reference with contraction off, so every value except the
// trigonometric ones (atan2 / sin / cos: the device libm, within an ulp of glibc) is bit-exact to
// sdf-nmpc_amd/ref_gen.py (tests/test_gpu_ref_pack.py).
#include <hip/hip_runtime.h>

#include <math.h>

#include "ref_kernels.h"

namespace sdfn {

namespace {

__device__ __forceinline__ double quat2yaw(const double* q) {  // utils/math.py:73-82
#pragma clang fp contract(off)
    return atan2(2 * (q[0] * q[3] + q[1] * q[2]), 1 - 2 * (q[2] * q[2] + q[3] * q[3]));
}
__device__ __forceinline__ void yaw2quat(double yaw, double* q) {  // utils/math.py:142-166
    const double h = yaw * 0.5;
    q[0] = cos(h);
    q[1] = 0.0;
    q[2] = 0.0;
    q[3] = sin(h);
}
__device__ __forceinline__ double norm3(double a, double b, double c) {
#pragma clang fp contract(off)
    return sqrt(a * a + b * b + c * c);
}
__device__ __forceinline__ double norm2(double a, double b) {
#pragma clang fp contract(off)
    return sqrt(a * a + b * b);
}

}  // namespace

__global__ __launch_bounds__(64) void ref_pack_kernel(RefPackArgs A) {
#pragma clang fp contract(off)
    const int b = blockIdx.x, tid = threadIdx.x, N = A.N, N1 = N + 1, np_ = A.np_, ny = A.ny;
    const double* x0 = A.x0 + (size_t)b * A.x0_stride;
    double* P = A.p + (size_t)b * N1 * np_;

    // ---- set_latent / set_sdf_flag (controller.py:45-54): every node
    if (A.latent) {
        const double* Rb = A.W_R_Bo + (size_t)b * 9;
        const double* pb = A.W_p_Bo + (size_t)b * 3;
        double pc[3], rc[9];
        for (int i = 0; i < 3; ++i) {  // W_R_Bo @ B_p_C + W_p_Bo
            pc[i] = (Rb[i * 3 + 0] * A.B_p_C[0] + Rb[i * 3 + 1] * A.B_p_C[1] + Rb[i * 3 + 2] * A.B_p_C[2]) + pb[i];
            for (int j = 0; j < 3; ++j)  // (W_R_Bo @ B_R_C).reshape(9), row-major
                rc[i * 3 + j] = Rb[i * 3 + 0] * A.B_R_C[0 * 3 + j] + Rb[i * 3 + 1] * A.B_R_C[1 * 3 + j] +
                                Rb[i * 3 + 2] * A.B_R_C[2 * 3 + j];
        }
        for (int k = tid; k < N1; k += 64) {
            double* pk = P + (size_t)k * np_;
            if (A.flag) pk[0] = A.flag[b];
            for (int i = 0; i < 3; ++i) pk[1 + i] = pc[i];
            for (int i = 0; i < 9; ++i) pk[4 + i] = rc[i];
        }
        const double* lat = A.latent + (size_t)b * A.L;
        for (int e = tid; e < N1 * A.L; e += 64) {
            const int k = e / A.L, j = e - k * A.L;
            P[(size_t)k * np_ + 17 + j] = lat[j];
        }
    } else if (A.flag) {
        for (int k = tid; k < N1; k += 64) P[(size_t)k * np_] = A.flag[b];
    }
    if (A.mode < 0) return;  // latent / flag only

    // ---- the reference trajectory (ref_gen.py)
    const int nw = A.n_wp, npt = nw + 1;
    const double* wpp = A.wp_p + (size_t)b * nw * 3;
    const double* wpq = A.wp_q + (size_t)b * nw * 4;
    auto Pp = [&](int i, int c) { return i == 0 ? x0[c] : wpp[(i - 1) * 3 + c]; };
    auto Pq = [&](int i, int c) { return i == 0 ? x0[3 + c] : wpq[(i - 1) * 4 + c]; };
    double q0[4] = {x0[3], x0[4], x0[5], x0[6]};

    int count = N1;            // references produced (N for from_x0 and stop-and-turn)
    int kind = 0;              // 0 path samples, 1 constant (hover / stop-and-turn), 2 joystick
    double cp[3] = {0, 0, 0}, cq[4] = {1, 0, 0, 0}, cv[3] = {0, 0, 0}, cwz = 0.0;
    double cum[RP_MAX_WP + 1], dist[RP_MAX_WP];
    double vref_e = 0.0, step = 0.0;
    int n_even = 0;
    if (A.mode == 2) {  // from_x0 (ref_gen.py:17-23)
        kind = 1;
        count = N;
        for (int c = 0; c < 3; ++c) cp[c] = x0[c];
        yaw2quat(quat2yaw(q0), cq);
    } else if (A.mode == 1) {  // gen_ref_joystick (ref_gen.py:101-130)
        kind = 2;
        const double* vw = A.vw + (size_t)b * 4;
        for (int c = 0; c < 3; ++c) cv[c] = vw[c] * A.vref;
        cwz = vw[3] * A.wzref;
        if (A.yaw_mode == 3) {
            yaw2quat(quat2yaw(q0), cq);
        } else if (A.yaw_mode == 2) {
            if (norm2(cv[0], cv[1]) > A.dmin) yaw2quat(atan2(cv[1], cv[0]), cq);
            else yaw2quat(quat2yaw(q0), cq);
        }
    } else {  // gen_ref_list_wps (ref_gen.py:25-99)
        bool stop = false;
        if (A.st_enable) {
            const double yaw_curr = quat2yaw(q0);
            double yaw_r = yaw_curr;
            if (A.st_mode == 1) {
                double q1[4] = {Pq(1, 0), Pq(1, 1), Pq(1, 2), Pq(1, 3)};
                yaw_r = quat2yaw(q1);
            } else if (A.st_mode == 2) {
                const double dx = Pp(1, 0) - x0[0], dy = Pp(1, 1) - x0[1];
                if (norm2(dx, dy) > A.dmin) yaw_r = atan2(dy, dx);
                yaw_r += A.align_off;
            }
            if (fabs(yaw_curr - yaw_r) > A.st_dang) {
                stop = true;
                kind = 1;
                count = N;
                for (int c = 0; c < 3; ++c) cp[c] = x0[c];
                yaw2quat(yaw_r, cq);
            }
        }
        if (!stop) {
            cum[0] = 0.0;
            for (int s = 0; s < nw; ++s) {
                dist[s] = norm3(Pp(s + 1, 0) - Pp(s, 0), Pp(s + 1, 1) - Pp(s, 1), Pp(s + 1, 2) - Pp(s, 2));
                cum[s + 1] = cum[s] + dist[s];
            }
            const double total = cum[nw];
            if (total / 1e-3 != 0.0) {
                vref_e = A.vref < total ? A.vref : total;
                step = A.T / N * vref_e;
                const double ne = ceil(total / step);  // numpy.arange length
                n_even = ne > (double)N1 ? N1 : (int)ne;
            }
        }
    }

    // node k's sample along the path (k < n_even)
    auto sample = [&](int k, double* p, double* q, double* v) {
        const double d = (double)k * step;
        int idx = 0;  // searchsorted(cum, d) (side='left')
        while (idx < npt && cum[idx] < d) ++idx;
        int s = idx - 1;
        s = s < 0 ? 0 : (s > nw - 1 ? nw - 1 : s);
        const double dd = d - cum[s];
        for (int c = 0; c < 3; ++c) {
            const double dir = (Pp(s + 1, c) - Pp(s, c)) / dist[s];
            p[c] = Pp(s, c) + dir * dd;
            v[c] = dir * vref_e;
        }
        if (A.yaw_mode == 3) {
            for (int c = 0; c < 4; ++c) q[c] = q0[c];
        } else if (A.yaw_mode == 1) {
            double qs[4] = {Pq(s + 1, 0), Pq(s + 1, 1), Pq(s + 1, 2), Pq(s + 1, 3)};
            yaw2quat(quat2yaw(qs), q);
        } else if (A.yaw_mode == 2) {
            if (norm2(Pp(1, 0) - x0[0], Pp(1, 1) - x0[1]) > A.dmin) {
                double yaw_r = atan2(v[1], v[0]);
                yaw_r += A.align_off;
                yaw2quat(yaw_r, q);
            } else {
                for (int c = 0; c < 4; ++c) q[c] = q0[c];
            }
        } else {
            q[0] = 1.0; q[1] = 0.0; q[2] = 0.0; q[3] = 0.0;
        }
    };

    for (int k = tid; k < count; k += 64) {
        double p[3], q[4], v[3] = {0, 0, 0}, wz = 0.0;
        if (kind == 1) {
            for (int c = 0; c < 3; ++c) p[c] = cp[c];
            for (int c = 0; c < 4; ++c) q[c] = cq[c];
        } else if (kind == 2) {
            for (int c = 0; c < 3; ++c) {
                p[c] = x0[c] + cv[c] * (double)k * A.T / N;
                v[c] = cv[c];
            }
            for (int c = 0; c < 4; ++c) q[c] = cq[c];
            wz = cwz;
        } else if (k < n_even) {
            sample(k, p, q, v);
        } else {  // padding (ref_gen.py:94-98): last sample's p / q, or the path end; v = 0, wz = 0
            if (n_even > 0) {
                double vv[3];
                sample(n_even - 1, p, q, vv);
            } else {
                for (int c = 0; c < 3; ++c) p[c] = Pp(nw, c);
                for (int c = 0; c < 4; ++c) q[c] = Pq(nw, c);
            }
        }
        // set_ref (controller.py:133-142) with formate_ref's layout
        double* pk = P + (size_t)k * np_;
        for (int c = 0; c < 4; ++c) pk[13 + c] = q[c];
        const double yr[11] = {p[0], p[1], p[2], 0.0, v[0], v[1], v[2], 0.0, 0.0, wz, 0.0};
        if (k < N) {
            double* yk = A.yref + ((size_t)b * N + k) * ny;
            double* wk = A.W + ((size_t)b * N + k) * ny;
            for (int i = 0; i < ny; ++i) {
                yk[i] = i < 11 ? yr[i] : 0.0;
                wk[i] = A.wrow[i];
            }
        } else {
            for (int i = 0; i < A.nyN; ++i) {  // yN = y[:nyN], WN = W[:nyN] (controller.py:141-142)
                A.yNref[(size_t)b * A.nyN + i] = yr[i];
                A.WN[(size_t)b * A.nyN + i] = A.wrow[i];
            }
        }
    }
}

hipError_t launch_ref_pack(const RefPackArgs& a, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    hipLaunchKernelGGL(ref_pack_kernel, dim3(a.B), dim3(64), 0, s, a);
    return hipGetLastError();
}

}  // namespace sdfn
