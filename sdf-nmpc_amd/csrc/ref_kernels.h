// Batched reference / parameter packing (ref_pack.hip): argument block shared with the engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace sdfn {

constexpr int RP_MAX_WP = 32;  // waypoints per instance

struct RefPackArgs {
    int B, N, np_, ny, n_wp, L;
    int nyN;  // terminal residual rows (4, or 5 with flags.stability)
    int mode;                      // 0 gen_ref_list_wps, 1 gen_ref_joystick, 2 from_x0, -1 latent / flag only
    int yaw_mode;                  // path samples: 0 identity, 1 'ref', 2 'align', 3 x0 quaternion ('curent')
    int st_enable, st_mode;        // stop-and-turn; st_mode 0 current yaw, 1 'topic', 2 'align'
    double st_dang, align_off, dmin, vref, wzref, T;
    double B_p_C[3], B_R_C[9];
    const double* x0;
    int x0_stride;
    const double *wp_p, *wp_q, *vw, *wrow;
    const double *latent, *W_p_Bo, *W_R_Bo, *flag;
    double *p, *yref, *W, *yNref, *WN;
};

hipError_t launch_ref_pack(const RefPackArgs& a, hipStream_t s);

}  // namespace sdfn
