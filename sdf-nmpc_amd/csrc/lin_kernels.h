// Shared definitions of the fp64 linearisation kernels (linearize.hip) and the engine.
#pragma once
#include <hip/hip_runtime.h>

namespace sdfn {

// 'att' quadrotor model constants (quad_rollpitchyawrate.py, default.yaml robot.limits / sensor)
struct QuadModel {
    double gamma, roll, pitch, wz;  // input scalings u -> (thrust/m, roll, pitch, yaw rate)
    double g;                       // 9.81 (base_model.py:10)
    double fov_off[3];              // B_R_C^T B_p_C + [fov_const_offset, 0, 0] (cost_const_helpers.py:64-65)
    double max_df;                  // NeuralDF.max_df: h_sdf when flag = 0 (gen_model.py:61)
    double B_R_C[9];                // sensor.B_R_C row-major (the Co_p_E rows of rec_feas)
    int rec_feas, stability;        // terminal extras (include/sdfnmpc.h sdfnmpc_quad_model)
    int poly_deg;                   // braking-distance polynomial (utils/math.py:294-321)
    double poly[84];
};

struct LinArgs {
    const double* x;   // [B][N+1][10]
    const double* u;   // [B][N][4]
    const double* p;   // [B][N+1][np]
    const double* dt;  // [N]
    double* xn;        // [B][N][10]
    double* AB;        // [B][N][14][10]   column j = d x_{k+1} / d (x,u)_j
    double* y;         // [B][N][11]
    double* Jy;        // [B][N][14][11]
    double* yN;        // [B][nyN]
    double* JyN;       // [B][10][nyN]
    double* h;         // [B][N+1][3]      rows 0,1 (row 2: sdf_mlp_kernel)
    double* Jh;        // [B][N+1][10][3]  rows 0,1
    double* hE;        // [B][6]           terminal extras (m.rec_feas / m.stability), else unused
    double* JhE;       // [B][10][6]
    QuadModel m;
    int B, N, np, nyN;
};

hipError_t launch_linearize(const LinArgs& a, hipStream_t s);

}  // namespace sdfn
