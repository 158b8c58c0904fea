/* boda_hip_vendor.h -- same-node comparator library (libboda_hip_vendor.so): rocBLAS SGEMM and
 * MIOpen convolution forward on the hot path's op shapes, for a per-op vendor time beside the
 * hand-written kernels of libboda_hip.so. It plays the role of the reference's culibs-wrap
 * intercepts (cublas_sgemm / cudnn_conv, src/culibs-wrap.cc:94-242) as cnn_op_info's use_culibs
 * comparator runs them (src/cnn-prof.cc:40,90-91). Context only: the product never links it.
 *
 * Operand layouts are those of boda_hip.h (bh_sgemm_kmajor, bh_conv2d_fwd_nchw), so a caller can
 * run both libraries on the same device buffers. Each context has its own HIP stream. */
#ifndef BODA_HIP_VENDOR_H
#define BODA_HIP_VENDOR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BHV_OK 0
#define BHV_ERR 1

typedef struct bhv_ctx bhv_ctx;

const char *bhv_last_error(void);
int bhv_init(int device, bhv_ctx **ctx);
int bhv_destroy(bhv_ctx *ctx);
int bhv_sync(bhv_ctx *ctx);

/* c[m][n] = sum_k a[k][m] * b[k][n] through rocblas_sgemm (as bh_sgemm_kmajor) */
int bhv_sgemm_kmajor(bhv_ctx *ctx, const float *a, const float *b, float *c, uint32_t M, uint32_t N, uint32_t K);

/* MIOpen conv forward (its Find choice, cached per shape), + bias (miopenOpTensor) + optional
 * ReLU (miopenActivationForward), operands as bh_conv2d_fwd_nchw */
int bhv_conv2d_fwd_nchw(bhv_ctx *ctx, const float *in, const float *filts, const float *biases, float *out,
                        uint32_t B, uint32_t IC, uint32_t H, uint32_t W, uint32_t OC, uint32_t KY, uint32_t KX,
                        uint32_t sy, uint32_t sx, uint32_t py, uint32_t px, int relu);

/* per-call milliseconds over `reps` back-to-back calls on internal operands (HIP events around
 * the run, one warm call before it). bhv_time_conv also reports the conv-only time (no bias, no
 * ReLU; may be NULL), the one-off Find time and MIOpen's algorithm family. */
int bhv_time_sgemm(bhv_ctx *ctx, uint32_t M, uint32_t N, uint32_t K, int reps, float *ms);
int bhv_time_conv(bhv_ctx *ctx, uint32_t B, uint32_t IC, uint32_t H, uint32_t W, uint32_t OC, uint32_t KY,
                  uint32_t KX, uint32_t sy, uint32_t sx, uint32_t py, uint32_t px, int relu, int reps, float *ms,
                  float *conv_only_ms, float *find_ms, char *algo, size_t algolen);

#ifdef __cplusplus
}
#endif

#endif
