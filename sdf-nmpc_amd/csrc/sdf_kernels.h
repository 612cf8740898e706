// Shared definitions of the SDF kernels (sdf_mlp.hip) and their host launchers (engine.cpp).
// Architecture: the deployed NeuralDF (scripts/neural_nets/df_train.py:98-102):
// embed 'oct', nb_freqs 5, latent 128, layer_sizes [256, 256, 128, 64], res 'full'.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace sdfn {

constexpr int EMB_ND = 8, EMB_NF = 5;
constexpr int EMB_NB = EMB_ND * EMB_NF;  // 40 projected frequencies
constexpr int E = 3 + 2 * EMB_NB;        // 83 embedding features (embeddings.py:104)
constexpr int KE = 88;                   // E padded to a multiple of 8 (MFMA k-grouping)
constexpr int NE = 96;                   // E padded to 3 column blocks of 32 (d e GEMM)
constexpr int L = 128;                   // latent size (default.yaml nn.size_latent)
constexpr int N1 = 256, N2 = 256, N3 = 128, N4 = 64;
constexpr int C13_STRIDE = N1 + N3;      // hoisted [c1 | c3] per instance
constexpr int SE = 92;                   // LDS row strides (floats): stride/4 odd -> conflict-free b128
constexpr int SA = 260;

// Packed operand: OUT[M x N] = IN[M x K] . Wsrc^T, Wsrc(j, k) = weight of output j, input k.
// Layout [cb][g][lane][4] with value Wsrc(cb*32 + (lane&31), (lane>>5)*K/2 + 4g + i), zero-padded.
inline size_t packed_floats(int N, int K) { return (size_t)((N + 31) / 32) * (K / 8) * 64 * 4; }

struct SdfArgs {
    // forward operands
    const float4* wF1;   // W1[:, :E]            N1 x KE
    const float4* wF2;   // W2                   N2 x N1
    const float4* wF3h;  // W3[:, :N2]           N3 x N2
    const float4* wF3e;  // W3[:, N2:N2+E]       N3 x KE
    const float4* wF4;   // W4                   N4 x N3
    // backward operands (transposed)
    const float4* wB4;   // W4^T                 N3 x N4
    const float4* wB3;   // W3[:, :N2]^T         N2 x N3
    const float4* wB3e;  // W3[:, N2:N2+E]^T     NE x N3
    const float4* wB2;   // W2^T                 N1 x N2
    const float4* wB1e;  // W1[:, :E]^T          NE x N1
    const float4* wB3z;  // W3[:, N2+E:]^T       L x N3   (latent gradient only)
    const float4* wB1z;  // W1[:, E:]^T          L x N1   (latent gradient only)
    const float* b2;
    const float* b4;
    const float* w5;
    const float4* emb_tab;  // [NE] (dirs[:, d] * 2^f) for m in the sin/cos ranges, else 0
    const float* c13;       // [n_inst][C13_STRIDE]
    const float4* pos;      // [rows] (Co_p_B as fp32, pad)           -- or, when x != NULL:
    const double* x;        // [rows][10] iterate; Co_p_B = W_R_Co^T (x[0:3] - W_p_Co) from p (fp64 -> fp32)
    float4* out;            // [rows] (df, d df/d pos)
    float* grad_latent;     // [rows][L] (latent-gradient variant only)
    // optional fused constraint epilogue (sdfnmpc_linearize): h[r][2] = flag df + (1 - flag) max_df,
    // Jh[r][j][2] = flag (d df / d Co_p_B) W_R_Co^T (j < 3), 0 (j >= 3)   -- gen_model.py:46-61
    const double* p;        // [rows][np] stage parameters (flag at 0, W_R_Co row-major at 4..12)
    double* h;              // [rows][3]      (NULL: no constraint epilogue)
    double* Jh;             // [rows][10][3]
    double max_df;
    int np;
    float b5;
    float w0;
    int rows;
    int rows_per_inst;      // row r uses c13[r / rows_per_inst]
};

// single-row latency path (sdf_row.hip): plain row-major torch-layout weights, value + full input gradient
struct SdfRowArgs {
    const float *W1, *b1;   // [N1][E + L], [N1]     (rows padded to a multiple of 4 floats)
    const float *W2, *b2;   // [N2][N1]
    const float *W3, *b3;   // [N3][N2 + E + L]
    const float *W4, *b4;   // [N4][N3]
    const float *W1T, *W2T, *W3T, *W4T;  // the same, transposed ([K][J]): the forward's coalesced operand
    const float* w5;        // [N4]
    float b5, w0;
    const float4* emb_tab;  // [NE]
    const float4* pos;      // [rows] (Co_p_B, pad)
    const float* latent;    // [rows][L]
    float4* out;            // [rows] (df, d df / d pos)
    float* grad_latent;     // [rows][L] or NULL
    int rows;
    // preparation-phase variant (sdfnmpc_linearize at a few rows, x != NULL): Co_p_B from x / p and the
    // constraint epilogue exactly as sdf_mlp_kernel forms them (SdfArgs), the latent from the fp64
    // stage parameters of the row's instance
    const double *x, *p;    // [rows][10], [rows][np]
    const double* zd;       // latent of row r at zd[(r / rows_per_inst) * zstride + k]
    long long zstride;
    int np, rows_per_inst;
    double *h, *Jh;         // [rows][3], [rows][10][3]: the sdf row
    double max_df;
    long long* stamps;      // diagnostics: phase wall-clock stamps (the server), or NULL
};
constexpr int SDF_ROW_MAX = 16;       // host-path calls with at most this many rows use sdf_row_kernel
constexpr int SDF_ROW_PREP_MAX = 64;  // and preparation phases with at most this many rows (B=1 at N <= 63)

// Resident SDF server (the C2 latency path, sdf_row.hip): one persistent workgroup polls this mailbox in
// pinned, coherent host memory, so a CasADi-external call costs no kernel launch and no copies.  The host
// writes rows / grad / in, then seq_in (release); the server stages the request into LDS, evaluates the
// rows with sdf_row's arithmetic, writes out, then seq_out = seq_in (release).  The server exits on
// `stop`, after `idle` wall-clock ticks without a request, or after `life` ticks in total; the host
// relaunches it when it finds it gone.  Sequence words sit on their own 128-byte lines.
struct alignas(128) SdfMbox {
    unsigned long long seq_in;
    unsigned long long pad0[15];
    unsigned long long seq_out;
    unsigned long long pad1[15];
    unsigned long long stop;
    unsigned long long gone;             // the server writes its launch epoch here when it exits
    int rows, grad;
    long long t_seen, t_staged, t_done;  // server wall-clock stamps of the last request (diagnostics)
    unsigned long long pad2[10];
    long long t_phase[16];               // row_eval's phase stamps of the last request (diagnostics)
    float in[SDF_ROW_MAX * (4 + 128)];   // [rows][4] Co_p_B | [rows][L] latent
    float out[SDF_ROW_MAX * (4 + 128)];  // [rows][4] (df, d df / d pos) | [rows][L] d df / d latent
};
constexpr int SDF_MBOX_FLOATS = SDF_ROW_MAX * (4 + 128);  // in / out capacity (rows x (4 + size_latent))

template <typename T>
struct HoistArgs {
    const T* latent;     // latent of instance i at latent[i * stride + k]
    long long stride;
    const float4* wpk;   // packed operand Wsrc(j, k) = [W1[:, E:] ; W3[:, N2+E:]](j, k), N = C13_STRIDE, K = L
    const float* bias;   // [C13_STRIDE] = [b1 | b3]
    float* c13;          // [n_inst][C13_STRIDE]
    int n_inst;
};
constexpr int HOIST_ROWS = 32;                    // instances per hoist workgroup (one MFMA row block)
constexpr int HOIST_COLS = 128;                   // output columns per hoist workgroup (4 waves x 32)
constexpr int SZ = L + 4;                         // LDS row stride of the latent tile

// ---- wide networks (layer sizes multiples of 128, e.g. C5's [1024,1024,512,256]): sdf_wide.hip
enum { WIDE_EPI_SIN = 0, WIDE_EPI_SIN_L4 = 1, WIDE_EPI_BWD = 2, WIDE_EPI_STORE = 3 };

// out[M x N] = [A1 | A2][M x (K1 + K2)] . W^T,  W [N][K1 + K2] row-major (K contiguous)
struct WideGemmArgs {
    const float* A1; int lda1, K1;
    const float* A2; int lda2, K2;   // optional second K segment (A2 = NULL, K2 = 0)
    const float* W;
    int M, N;
    const float* bias;               // [N] (SIN / SIN_L4 / STORE) or NULL
    const float* c; int ldc;         // per-instance additive term c[m / rows_per_inst][n] (SIN), or NULL
    int rows_per_inst;
    const float* d; int ldd;         // BWD: cos(w0 a) of the layer
    const float* w5;                 // SIN_L4: final-layer weights
    float* out1; int ld1;            // SIN: sin(w0 a) | BWD: ((acc * d) * w0) | STORE: acc + bias
    float* out2; int ld2;            // SIN: cos(w0 a) | SIN_L4: (w5 * cos(w0 a)) * w0  (act' for relu / softplus)
    float w0;
    int act;                         // 0 sin(w0 .), 1 relu, 2 softplus (neural_df.py:40-47)
};

struct WideSdfArgs {
    int rows, n4, np;
    int nb, nek, neb;                 // projected frequencies; E / G row stride; GE3 / GE1 row stride
    const double* x; const double* p;  // Co_p_B from the iterate (or pos when x == NULL)
    const float4* pos;
    const float4* emb_tab;
    float* E; float* G;               // [rows][nek]
    const float* H4;                  // [rows][n4]
    const float* GE3; const float* GE1;  // [rows][neb]
    const float* w5; float b5;
    float4* out;                      // [rows] (df, d df / d pos) or NULL
    double* h; double* Jh; double max_df;
};

// Single-row latency path for every network other than the deployed one (sdf_row_wide.hip): the wide
// schedule's row-major [N][K] operands (engine.cpp upload_wide) as GEMVs inside one 512-thread workgroup per
// row, value + full input gradient (d df / d pos and d df / d latent), served by the resident server or
// launched per call.  Same semantics as wide_gemm's layers (activations, res modes, padding).
struct WideRowArgs {
    const float *F1, *F2, *F3, *F4;            // forward [P1][NEK], [P2][P1], [P3][P2 (+ NEK)], [P4][P3]
    const float *B4, *B3h, *B3e, *B2, *B1e;    // backward [P3][P4], [P2][P3], [NEB][P3], [P1][P2], [NEB][P1]
    const float *Bz, *Hz, *bz, *b2, *b4, *w5;  // [LZ][P1 + P3], [P1 + P3][LZ], [P1 + P3], [P2], [P4], [P4]
    const float4* emb_tab;                     // [NEK]
    float b5, w0;
    int P1, P2, P3, P4, NEK, NEB, nb, LH, LZ, e3, act;
    // per call
    const float4* pos;      // [rows] (Co_p_B, pad)
    const float* latent;    // [rows][LH]
    float4* out;            // [rows] (df, d df / d pos)
    float* grad_latent;     // [rows][LH] or NULL
    int rows;
};
size_t wide_row_lds_bytes(const WideRowArgs& a);        // the evaluator's dynamic LDS
int wide_row_max_rows(int LH);                           // rows per server request (the mailbox's capacity)
hipError_t launch_sdf_row_wide(const WideRowArgs& a, hipStream_t s);
hipError_t launch_sdf_server_wide(const WideRowArgs& a, SdfMbox* mb_dev, long long idle_ticks, long long life_ticks,
                                  unsigned long long epoch, hipStream_t s);

hipError_t launch_wide_gemm(const WideGemmArgs& a, int epi, hipStream_t s);
template <typename T>  // double (stage parameters) or float
hipError_t launch_wide_latent(const T* lat, long long stride, int n_inst, int lh, int lz, float* z, hipStream_t s);
hipError_t launch_wide_emb(const WideSdfArgs& a, hipStream_t s);
hipError_t launch_wide_final(const WideSdfArgs& a, hipStream_t s);

size_t sdf_lds_bytes(int M);
hipError_t sdf_set_lds_limits();
hipError_t launch_sdf_mlp(const SdfArgs& a, int M, bool latent_grad, hipStream_t s);
hipError_t launch_sdf_row(const SdfRowArgs& a, hipStream_t s);
hipError_t launch_sdf_server(const SdfRowArgs& a, SdfMbox* mb_dev, long long idle_ticks, long long life_ticks,
                             unsigned long long epoch, hipStream_t s);
template <typename T>
hipError_t launch_hoist(const HoistArgs<T>& a, hipStream_t s);

}  // namespace sdfn
