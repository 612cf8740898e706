/* CPU restatement of the in-loop VAE encoder path -- TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may call this; the product
 * path (csrc/vae_enc.hip) never does.  Pinned to tests/golden/vae_golden.npz, which holds outputs of
 * the reference's own Encoder / preprocessing modules (tests/golden/make_golden.py: vae_golden).
 *
 * orc_vae_preprocess  -- sdf_nmpc/vae.py:15-24: ToDevice (float32 cast, preprocessing.py:263-276),
 *                        Reshape (bilinear resize, align_corners=False, preprocessing.py:99-112),
 *                        ClipDistance (preprocessing.py:84-96), Depth2Range (preprocessing.py:5-30),
 *                        all in fp32 in torch's order.
 * orc_vae_encode      -- Encoder.forward (network/vae.py:39-43): conv7x7/2 + ELU + maxpool3/2 +
 *                        ResBlock(64,2) ResBlock(128,2) ResBlock(256,2) ResBlock(512,1)
 *                        (network/resnet.py:27-56, BatchNorm in eval mode, dropout identity) +
 *                        AdaptiveAvgPool2d((2,2)) + Flatten + mean Linear.  Computed in fp64 from the
 *                        UNFOLDED fp32 parameters in Encoder.state_dict() order, so it is an independent
 *                        check of the kernels' BatchNorm folding.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* OpenMP threads of the conv layers (0: the runtime default); set by the CPU-baseline leg of bench.py */
static int g_vae_threads = 0;
void orc_vae_set_threads(int n) { g_vae_threads = n > 0 ? n : 0; }
#ifdef _OPENMP
#include <omp.h>
static int vae_threads(void) { return g_vae_threads > 0 ? g_vae_threads : omp_get_max_threads(); }
#else
static int vae_threads(void) { return 1; }
#endif

/* ---- preprocessing (fp32, torch order) ---- */
void orc_vae_preprocess(const void* img, int dtype, int Hi, int Wi, int H, int W, float clip_scale,
                        const float* yz, float* out) {
    float* src = (float*)malloc(sizeof(float) * (size_t)Hi * Wi);
    for (long i = 0; i < (long)Hi * Wi; ++i)
        src[i] = dtype == 1 ? (float)((const unsigned short*)img)[i] : ((const float*)img)[i];
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            float v;
            if (Hi == H && Wi == W) {
                v = src[(long)y * W + x];
            } else { /* upsample_bilinear2d, align_corners=False, scale = in/out in fp32 */
                const float sh = (float)Hi / (float)H, sw = (float)Wi / (float)W;
                float fy = sh * ((float)y + 0.5f) - 0.5f, fx = sw * ((float)x + 0.5f) - 0.5f;
                if (fy < 0.f) fy = 0.f;
                if (fx < 0.f) fx = 0.f;
                const int y0 = (int)fy, x0 = (int)fx;
                const int y1 = y0 + (y0 < Hi - 1), x1 = x0 + (x0 < Wi - 1);
                const float ly1 = fy - (float)y0, ly0 = 1.f - ly1, lx1 = fx - (float)x0, lx0 = 1.f - lx1;
                const float* r0 = src + (long)y0 * Wi;
                const float* r1 = src + (long)y1 * Wi;
                v = ly0 * (lx0 * r0[x0] + lx1 * r0[x1]) + ly1 * (lx0 * r1[x0] + lx1 * r1[x1]);
            }
            v = v / clip_scale;
            v = v < 0.f ? 0.f : (v > 1.f ? 1.f : v);
            if (yz) {
                v = v * yz[(long)y * W + x];
                v = v < 0.f ? 0.f : (v > 1.f ? 1.f : v);
            }
            out[(long)y * W + x] = v;
        }
    free(src);
}

/* ---- encoder (fp64, NCHW) ---- */
typedef struct {
    const float* p;
} cursor;

static const float* take(cursor* c, long n) {
    const float* r = c->p;
    c->p += n;
    return r;
}

/* out[co][oy][ox] = sum w[co][ci][ky][kx] in[ci][iy][ix] (+ bias) */
static void conv2d(const double* in, int C, int H, int W, const float* w, const float* bias, int Co, int K,
                   int S, int P, double* out, int Ho, int Wo) {
#pragma omp parallel for schedule(static) num_threads(vae_threads())
    for (int co = 0; co < Co; ++co) {
        double* o = out + (long)co * Ho * Wo;
        for (long i = 0; i < (long)Ho * Wo; ++i) o[i] = bias ? (double)bias[co] : 0.0;
        for (int ci = 0; ci < C; ++ci)
            for (int ky = 0; ky < K; ++ky)
                for (int kx = 0; kx < K; ++kx) {
                    const double wv = (double)w[(((long)co * C + ci) * K + ky) * K + kx];
                    const double* ip = in + (long)ci * H * W;
                    for (int oy = 0; oy < Ho; ++oy) {
                        const int iy = oy * S - P + ky;
                        if (iy < 0 || iy >= H) continue;
                        for (int ox = 0; ox < Wo; ++ox) {
                            const int ix = ox * S - P + kx;
                            if (ix < 0 || ix >= W) continue;
                            o[(long)oy * Wo + ox] += wv * ip[(long)iy * W + ix];
                        }
                    }
                }
    }
}

/* BatchNorm2d in eval mode: (x - m) / sqrt(v + eps) * g + b */
static void bnorm(double* x, int C, long HW, const float* g, const float* b, const float* m, const float* v) {
    for (int c = 0; c < C; ++c) {
        const double s = 1.0 / sqrt((double)v[c] + 1e-5);
        for (long i = 0; i < HW; ++i) x[c * HW + i] = ((x[c * HW + i] - (double)m[c]) * s) * (double)g[c] + (double)b[c];
    }
}

static void relu(double* x, long n) {
    for (long i = 0; i < n; ++i) x[i] = x[i] < 0.0 ? 0.0 : x[i];  /* torch.relu keeps a NaN */
}

/* ResBlock(size_in, stride), non-bottleneck (resnet.py:27-56) */
static double* resblock(const double* in, int C, int H, int W, int S, int bn, cursor* cur, int* Ho_, int* Wo_) {
    const int Co = C * S, Ho = (H + 2 - 3) / S + 1, Wo = (W + 2 - 3) / S + 1;
    const long HWo = (long)Ho * Wo;
    double* h = (double*)malloc(sizeof(double) * Co * HWo);
    double* o = (double*)malloc(sizeof(double) * Co * HWo);
    const float* w0 = take(cur, (long)Co * C * 9);
    const float* b0 = bn ? NULL : take(cur, Co);
    conv2d(in, C, H, W, w0, b0, Co, 3, S, 1, h, Ho, Wo);
    if (bn) {
        const float *g = take(cur, Co), *b = take(cur, Co), *m = take(cur, Co), *v = take(cur, Co);
        bnorm(h, Co, HWo, g, b, m, v);
    }
    relu(h, Co * HWo);
    const float* w1 = take(cur, (long)Co * Co * 9);
    const float* b1 = bn ? NULL : take(cur, Co);
    conv2d(h, Co, Ho, Wo, w1, b1, Co, 3, 1, 1, o, Ho, Wo);
    if (bn) {
        const float *g = take(cur, Co), *b = take(cur, Co), *m = take(cur, Co), *v = take(cur, Co);
        bnorm(o, Co, HWo, g, b, m, v);
    }
    if (S == 1) {
        for (long i = 0; i < Co * HWo; ++i) o[i] += in[i];
    } else {
        const float* ws = take(cur, (long)Co * C);
        const float* bs = bn ? NULL : take(cur, Co);
        conv2d(in, C, H, W, ws, bs, Co, 1, S, 0, h, Ho, Wo);
        if (bn) {
            const float *g = take(cur, Co), *b = take(cur, Co), *m = take(cur, Co), *v = take(cur, Co);
            bnorm(h, Co, HWo, g, b, m, v);
        }
        for (long i = 0; i < Co * HWo; ++i) o[i] += h[i];
    }
    relu(o, Co * HWo);
    free(h);
    *Ho_ = Ho;
    *Wo_ = Wo;
    return o;
}

/* pre: [B][H][W] preprocessed fp32; params: Encoder.state_dict() order without num_batches_tracked;
 * latent: [B][L] fp64.  stage_sums (optional, [64+128+256+512+512]): per-channel sums after the
 * maxpool and each block, for image 0 (the golden file's debugging aid). */
void orc_vae_encode(const float* pre, int B, int H, int W, const float* params, int L, int bn, double* latent,
                    double* stage_sums) {
    for (int b = 0; b < B; ++b) {
        cursor cur = {params};
        const int H1 = (H + 6 - 7) / 2 + 1, W1 = (W + 6 - 7) / 2 + 1;
        double* x = (double*)malloc(sizeof(double) * (long)H * W);
        for (long i = 0; i < (long)H * W; ++i) x[i] = (double)pre[(long)b * H * W + i];
        double* c1 = (double*)malloc(sizeof(double) * 64L * H1 * W1);
        const float* w = take(&cur, 64 * 49);
        const float* bb = take(&cur, 64);
        conv2d(x, 1, H, W, w, bb, 64, 7, 2, 3, c1, H1, W1);
        for (long i = 0; i < 64L * H1 * W1; ++i) c1[i] = c1[i] > 0.0 ? c1[i] : expm1(c1[i]); /* ELU(1) */
        const int H2 = (H1 + 2 - 3) / 2 + 1, W2 = (W1 + 2 - 3) / 2 + 1;
        double* mp = (double*)malloc(sizeof(double) * 64L * H2 * W2);
        for (int c = 0; c < 64; ++c) /* MaxPool2d(3, 2, 1): padding never wins */
            for (int oy = 0; oy < H2; ++oy)
                for (int ox = 0; ox < W2; ++ox) {
                    double m = -INFINITY;
                    for (int ky = 0; ky < 3; ++ky)
                        for (int kx = 0; kx < 3; ++kx) {
                            const int iy = oy * 2 - 1 + ky, ix = ox * 2 - 1 + kx;
                            if (iy < 0 || iy >= H1 || ix < 0 || ix >= W1) continue;
                            const double v = c1[((long)c * H1 + iy) * W1 + ix];
                            m = (v > m || v != v) ? v : m;  /* torch max_pool2d propagates a NaN */
                        }
                    mp[((long)c * H2 + oy) * W2 + ox] = m;
                }
        free(x);
        free(c1);
        int C = 64, h = H2, wd = W2, off = 0;
        if (stage_sums && b == 0) {
            for (int c = 0; c < C; ++c) {
                double s = 0.0;
                for (long i = 0; i < (long)h * wd; ++i) s += mp[(long)c * h * wd + i];
                stage_sums[off + c] = s;
            }
            off += C;
        }
        double* cur_map = mp;
        const int strides[4] = {2, 2, 2, 1};
        for (int k = 0; k < 4; ++k) {
            int Ho, Wo;
            double* o = resblock(cur_map, C, h, wd, strides[k], bn, &cur, &Ho, &Wo);
            free(cur_map);
            cur_map = o;
            C *= strides[k];
            h = Ho;
            wd = Wo;
            if (stage_sums && b == 0) {
                for (int c = 0; c < C; ++c) {
                    double s = 0.0;
                    for (long i = 0; i < (long)h * wd; ++i) s += cur_map[(long)c * h * wd + i];
                    stage_sums[off + c] = s;
                }
                off += C;
            }
        }
        /* AdaptiveAvgPool2d((2,2)): bin i spans [floor(i*h/2), ceil((i+1)*h/2)); Flatten -> c*4 + i*2 + j */
        double feat[2048];
        for (int c = 0; c < C; ++c)
            for (int i = 0; i < 2; ++i)
                for (int j = 0; j < 2; ++j) {
                    const int y0 = (i * h) / 2, y1 = ((i + 1) * h + 1) / 2, x0 = (j * wd) / 2, x1 = ((j + 1) * wd + 1) / 2;
                    double s = 0.0;
                    for (int y = y0; y < y1; ++y)
                        for (int x = x0; x < x1; ++x) s += cur_map[((long)c * h + y) * wd + x];
                    feat[c * 4 + i * 2 + j] = s / (double)((y1 - y0) * (x1 - x0));
                }
        free(cur_map);
        const float* mw = take(&cur, (long)L * 2048);
        const float* mb = take(&cur, L);
        for (int o = 0; o < L; ++o) {
            double s = (double)mb[o];
            for (int f = 0; f < 2048; ++f) s += (double)mw[(long)o * 2048 + f] * feat[f];
            latent[(long)b * L + o] = s;
        }
    }
}
