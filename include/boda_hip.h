/*
 * boda_hip.h -- C-ABI of the MI355X (gfx950) backend for Boda's per-op
 * Convolution / SGEMM hot path (libboda_hip.so).
 *
 * This is the drop-in seam. Boda reaches device code only through the
 * rtc_compute_t plugin (src/rtc_compute.H:35-97); its CUDA implementation is
 * nvrtc_compute_t (src/nvrtc_util.cc:174-395) and its vendor-library
 * intercept is culibs_wrap_t (src/culibs-wrap.cc:66-242, dispatched from
 * src/nvrtc_util.cc:369-372). A C++ hip_compute_t (boda-1_amd/host/) binds
 * these entry points one-for-one; INTEGRATION.md shows that binding and the
 * ctypes binding used by the tests.
 *
 * Conventions
 *   - every call returns BH_OK (0) on success, BH_ERR (1) on a runtime error
 *     (Boda maps it to rt_err, src/boda_base.H:98-105) or BH_UNSUP (2) for an
 *     unsupported shape/argument (Boda's unsup_err, which ops-prof records and
 *     skips, src/rtc_prof.cc:287-296). bh_last_error() returns a thread-local
 *     message for the most recent failure on the calling thread.
 *   - pointers are device pointers unless named host_*; sizes are bytes
 *     unless named in elements. All tensors are dense fp32, row-major
 *     (innermost dimension last), exactly Boda's reference layouts.
 *   - work is issued on the context's stream in call order; nothing blocks
 *     except bh_d2h, bh_sync and bh_elapsed_ms.
 *   - the product path has no CPU fallback: with no usable gfx950 device,
 *     bh_init fails with BH_ERR.
 */
#ifndef BODA_HIP_H
#define BODA_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BH_OK 0
#define BH_ERR 1
#define BH_UNSUP 2

#define BH_ABI_VERSION 3

typedef struct bh_ctx bh_ctx;

/* ---- version / errors ------------------------------------------------- */
int bh_abi_version(void);
const char *bh_last_error(void);

/* ---- device context: nvrtc_compute_t::init (src/nvrtc_util.cc:184-213),
 *      get_plat_tag (src/rtc_compute.H:46) ------------------------------ */
int bh_device_count(int *count);
int bh_init(int device, bh_ctx **ctx);
int bh_destroy(bh_ctx *ctx);
/* "hip:<device name>:<gcnArch>" e.g. "hip:AMD Instinct MI355X:gfx950" */
int bh_plat_tag(bh_ctx *ctx, char *buf, size_t buflen);
/* the hipStream_t work is issued on (opaque; for interop only) */
int bh_get_stream(bh_ctx *ctx, void **stream);

/* ---- vars: create_var_with_dims (zero-filled, src/nvrtc_util.cc:80-84),
 *      release_var, set_var_to_zero, copy_nda_to_var, copy_var_to_nda
 *      (src/rtc_compute.H:48-52,88-91) --------------------------------- */
int bh_alloc(bh_ctx *ctx, size_t bytes, void **dptr);
int bh_free(bh_ctx *ctx, void *dptr);
int bh_memset0(bh_ctx *ctx, void *dptr, size_t bytes);
int bh_h2d(bh_ctx *ctx, void *dptr, const void *host_src, size_t bytes);
int bh_d2h(bh_ctx *ctx, void *host_dst, const void *dptr, size_t bytes);

/* ---- sync / timing: finish_and_sync, get_dur (ms), release_per_call_id_data
 *      (src/rtc_compute.H:60-71; events per call src/nvrtc_util.cc:289-298) */
int bh_sync(bh_ctx *ctx);
int bh_event_record(bh_ctx *ctx, int *event_id);
int bh_elapsed_ms(bh_ctx *ctx, int begin_id, int end_id, float *ms);
int bh_events_reset(bh_ctx *ctx);
/* arm an event pair for the NEXT hot-path / gen_data call on this context: its
 * first kernel dispatch records begin_id, its last records end_id, on the
 * dispatches themselves (hipExtLaunchKernel), so bh_elapsed_ms(begin, end) is the
 * call's GPU time (split-K reduce pass included) without host launch latency. */
int bh_time_next_call(bh_ctx *ctx, int *begin_id, int *end_id);
/* device timestamps, usable inside captured graphs: bh_stamp enqueues a write
 * of the GPU's constant-rate wall clock into slot (0 <= slot < 262144);
 * bh_stamps_read syncs and returns slots first..first+n-1 in microseconds
 * relative to slot first. */
int bh_stamp(bh_ctx *ctx, int slot);
int bh_stamps_read(bh_ctx *ctx, int first, int n, double *us);
/* enqueue a one-block kernel that busy-waits us microseconds (1..100000) on the
 * device clock: queued work behind it starts back to back, so events recorded
 * around a batch measure GPU time, not host launch latency. */
int bh_spin(bh_ctx *ctx, int us);

/* ---- launch batching: capture everything issued on the context between
 *      begin and end (kernels, event records) into a hipGraph and replay it
 *      with one call, so a sweep of small ops is not bound by host launch
 *      latency. Nothing may allocate while capturing (run one eager pass
 *      first so split-K workspaces exist). ---------------------------------- */
int bh_capture_begin(bh_ctx *ctx);
int bh_capture_end(bh_ctx *ctx, int *graph_id);
int bh_graph_launch(bh_ctx *ctx, int graph_id);
int bh_graph_destroy(bh_ctx *ctx, int graph_id);

/* ---- deterministic test data on the device: the gen_data_* kernels
 *      (test/rtc/gen-util.h:1-9, gen_data_sgemm_{a,b}.cucl,
 *      gen_data_Convolution_{in,filts,biases}.cucl; invoked from
 *      src/rtc_prof.cc:72-91). kind selects the template; d[] are the dims
 *      of the reference layout, outermost first (unused trailing dims = 1):
 *        BH_GEN_SGEMM_A   a  K:M         d = {K, M}
 *        BH_GEN_SGEMM_B   b  K:N         d = {K, N}
 *        BH_GEN_CONV_IN   in img:chan:y:x        d = {B, C, H, W}
 *        BH_GEN_CONV_FILTS filts out_chan:in_chan:y:x d = {OC, IC, KY, KX}
 *        BH_GEN_CONV_BIASES biases out_chan     d = {OC}
 *      mode: 2/3/4/5 as the templates, 600 (sgemm KAT), vi: added offset. */
#define BH_GEN_SGEMM_A 0
#define BH_GEN_SGEMM_B 1
#define BH_GEN_CONV_IN 2
#define BH_GEN_CONV_FILTS 3
#define BH_GEN_CONV_BIASES 4
int bh_gen_data(bh_ctx *ctx, int kind, float *dst, const uint32_t dims[4], uint32_t mode, float vi);

/* ---- the hot path ------------------------------------------------------
 * SGEMM: c[m][n] = sum_k a[k][m] * b[k][n]; a K x M, b K x N, c M x N.
 * Replaces the sgemm / sgemm_no_local / sgemm_simd / sgemm_simd_local CUCL
 * variants (test/rtc/sgemm*.cucl, generated by src/cnn_codegen.cc:293-490)
 * and the cublas_sgemm intercept (src/culibs-wrap.cc:214-242). Any M,N,K >= 1. */
int bh_sgemm_kmajor(bh_ctx *ctx, const float *a, const float *b, float *c,
                    uint32_t M, uint32_t N, uint32_t K);

/* Convolution forward, Caffe NCHW cross-correlation with symmetric zero
 * padding, fused per-output-channel bias and optional ReLU:
 *   out[n][oc][y][x] = act(biases[oc] + sum in[n][ic][y*sy+ky-py][x*sx+kx-px]
 *                                         * filts[oc][ic][ky][kx])
 * in B x IC x H x W, filts OC x IC x KY x KX, biases OC (may be NULL),
 * out B x OC x OH x OW with OH = (H + 2py - KY)/sy + 1 (src/conv_util.cc:167-173).
 * Replaces conv / tconv / k1conv / ipconv / conv_simd / k1conv_simd
 * (test/rtc/{conv,tconv,k1conv,ipconv}.cucl etc., selected by src/cnn_op.cc:16-331) and the cudnn_conv
 * intercept (src/culibs-wrap.cc:94-212). ReLU is what ops-prof always fuses
 * (conv_has_relu=1, src/cnn_op.cc:335-337). The variant is chosen per shape;
 * bh_variant_name reports which one runs. */
int bh_conv2d_fwd_nchw(bh_ctx *ctx, const float *in, const float *filts, const float *biases,
                       float *out, uint32_t B, uint32_t IC, uint32_t H, uint32_t W,
                       uint32_t OC, uint32_t KY, uint32_t KX, uint32_t sy, uint32_t sx,
                       uint32_t py, uint32_t px, int relu);

/* Filter-bank transform for the conv variants that read the filters k-major --
 * Boda's xpose_filts (test/rtc/xpose_filts.cucl, run once per var before the
 * timed calls: src/rtc_prof.cc:93-99, src/rtc_fwd.cc:306-326). A pack is, in order:
 *  - the k-major bank: row (ky*KX+kx)*IC + ic holds filts[*][ic][ky][kx] for every output
 *    channel, ceil4(OC) floats per row, ceil64(IC*KY*KX) rows (the padding rows zero);
 *  - then the Winograd banks its mask names, in bit order (each only for its kernel size):
 *      BH_BANK_W23  3x3, F(2x2,3x3): U = G g G^T, [ceil4(IC)][ceil32(OC)][16] floats, each
 *                   (ic, oc) row's four 4-float chunks rotated by (oc >> 2) & 3;
 *      BH_BANK_W43  3x3, F(4x4,3x3): U = G g G^T over points 0, +-2/3, +-3/2, infinity, made in
 *                   double and rounded once, [ceil4(IC)][ceil32(OC)][36] floats, the 36
 *                   positions in the position-split kernels' (group, slot) order;
 *      BH_BANK_W25  5x5, F(2x2,5x5): the same form and layout as W43 for the 5x5 filter.
 * bh_conv_filts_pack / bh_conv_filts_packed_floats make the FULL pack (mask BH_BANKS_ALL: a 3x3's
 * k-major + W23 + W43 = 6.8x the filter bytes, a 5x5's k-major + W25 = 2.4x, other kernels the
 * k-major bank alone), which bh_conv2d_fwd_nchw_pk / _res / _slab read: any route of the shape
 * finds its bank there. ABI 3 adds packs of chosen banks: bh_conv_route_banks names the bank the
 * shape's route reads now (0: none), bh_conv_filts_pack_banks makes a pack of exactly those, and
 * bh_conv2d_fwd_nchw_pkb takes the mask with the pack. A route whose bank a pack lacks makes it
 * inside the call (correct, slower). */
#define BH_BANK_W23 1u
#define BH_BANK_W43 2u
#define BH_BANK_W25 4u
#define BH_BANKS_ALL 0xffffffffu
size_t bh_conv_filts_packed_floats(uint32_t OC, uint32_t IC, uint32_t KY, uint32_t KX);
int bh_conv_filts_pack(bh_ctx *ctx, const float *filts, float *packed, uint32_t OC, uint32_t IC,
                       uint32_t KY, uint32_t KX);
size_t bh_conv_filts_packed_floats_banks(uint32_t OC, uint32_t IC, uint32_t KY, uint32_t KX, uint32_t banks);
int bh_conv_filts_pack_banks(bh_ctx *ctx, const float *filts, float *packed, uint32_t OC, uint32_t IC,
                             uint32_t KY, uint32_t KX, uint32_t banks);
/* *banks = the Winograd bank (BH_BANK_*) the route of conv shape dims[0..10] = B,IC,H,W,OC,KY,KX,
 * sy,sx,py,px reads on ctx now (its tuning table / overrides), 0 for a route of the k-major bank;
 * ctx may be NULL (the tuning table's / heuristic's route, no device needed) */
int bh_conv_route_banks(bh_ctx *ctx, const uint32_t *dims, uint32_t *banks);
/* bh_conv2d_fwd_nchw with the transformed bank of filts already made by
 * bh_conv_filts_pack (packed may be NULL: then a variant that needs it makes it
 * itself, inside the call). filts must still be given: variants that read the
 * reference layout use it. */
int bh_conv2d_fwd_nchw_pk(bh_ctx *ctx, const float *in, const float *filts, const float *packed,
                          const float *biases, float *out, uint32_t B, uint32_t IC, uint32_t H,
                          uint32_t W, uint32_t OC, uint32_t KY, uint32_t KX, uint32_t sy,
                          uint32_t sx, uint32_t py, uint32_t px, int relu);
/* bh_conv2d_fwd_nchw_pk writing channels out_chan_ofs .. out_chan_ofs+OC-1 of an output
 * tensor B x out_chans_total x OH x OW (out points at its start): a conv whose only reader is
 * a Concat writes its slab of the Concat's output in place, so the net executor runs no
 * channel copy for it (the reference's conv_pipe_fwd_t copies every Concat input with
 * copy.cucl, src/rtc_fwd.cc:267-280). */
/* bh_conv2d_fwd_nchw_pk with a residual: out = relu?(conv + bias + res), res B x OC x OH x OW
 * (may be NULL; may not overlap out unless equal to it). The add is the conv's epilogue, in the
 * order of a separate Caffe Eltwise SUM of the stored conv output and res (bit-identical to
 * it): the net executor folds a ResNet shortcut Eltwise (+ its ReLU) into the conv producing
 * one of its inputs. The reference runs Eltwise as its own layer only in Caffe (its rtc_fwd
 * rejects it, src/rtc_fwd.cc:404). */
int bh_conv2d_fwd_nchw_res(bh_ctx *ctx, const float *in, const float *filts, const float *packed,
                           const float *biases, const float *res, float *out, uint32_t B, uint32_t IC,
                           uint32_t H, uint32_t W, uint32_t OC, uint32_t KY, uint32_t KX, uint32_t sy,
                           uint32_t sx, uint32_t py, uint32_t px, int relu);
int bh_conv2d_fwd_nchw_slab(bh_ctx *ctx, const float *in, const float *filts, const float *packed,
                            const float *biases, float *out, uint32_t out_chans_total,
                            uint32_t out_chan_ofs, uint32_t B, uint32_t IC, uint32_t H, uint32_t W,
                            uint32_t OC, uint32_t KY, uint32_t KX, uint32_t sy, uint32_t sx,
                            uint32_t py, uint32_t px, int relu);
/* ABI 3, every conv form in one call: packed (may be NULL) holds the k-major bank + the Winograd
 * banks of mask `banks` (bh_conv_filts_pack_banks; BH_BANKS_ALL: bh_conv_filts_pack's layout);
 * res (may be NULL) as _res; the output a channel slab out_chan_ofs .. +OC-1 of a tensor of
 * out_chans_total channels (0: OC) as _slab (not together with res). */
int bh_conv2d_fwd_nchw_pkb(bh_ctx *ctx, const float *in, const float *filts, const float *packed, uint32_t banks,
                           const float *biases, const float *res, float *out, uint32_t out_chans_total,
                           uint32_t out_chan_ofs, uint32_t B, uint32_t IC, uint32_t H, uint32_t W, uint32_t OC,
                           uint32_t KY, uint32_t KX, uint32_t sy, uint32_t sx, uint32_t py, uint32_t px, int relu);

/* ---- the other forward layers of Boda's net executor (conv_pipe_fwd_t::gen_op,
 *      src/rtc_fwd.cc:263-405), NCHW fp32 ------------------------------------ */
/* Pooling (test/rtc/pool.cucl; Caffe output size, a partial last window adds an
 * output: src/conv_util.cc:198-204): max (avg=0) or average (avg=1) over the
 * in-image taps of each KY x KX window. out_in_yx (may be NULL): max pooling's
 * winning in_y*W+in_x per output, as float (-1: none). Global pooling: KY=H,
 * KX=W, strides 1, no padding. */
int bh_pool_out_size(uint32_t in, uint32_t k, uint32_t stride, uint32_t pad);
int bh_pool_fwd_nchw(bh_ctx *ctx, const float *in, float *out, float *out_in_yx, uint32_t B, uint32_t C,
                     uint32_t H, uint32_t W, uint32_t KY, uint32_t KX, uint32_t sy, uint32_t sx, uint32_t py,
                     uint32_t px, int avg);
/* LRN across channels (test/rtc/lrn.cucl, Caffe-matching running sum):
 * out = in * (k + alpha/local_size * sum of squares over local_size channels)^-beta;
 * out_scale_base (may be NULL) receives the base. local_size odd, <= 11. */
int bh_lrn_fwd_nchw(bh_ctx *ctx, const float *in, float *out, float *out_scale_base, uint32_t B, uint32_t C,
                    uint32_t H, uint32_t W, uint32_t local_size, float alpha, float beta, float k);
/* ReLU in place (test/rtc/relu.cucl); x 16-byte aligned, n elements. */
int bh_relu_inplace(bh_ctx *ctx, float *x, uint64_t n);
/* Deterministic dropout in place (test/rtc/dropout.cucl; the rtc mode's Dropout, seeded by
 * has_conv_fwd_t::set_det_drop_seed, src/rtc_fwd.cc:91-99,348-358): x[i] = murmur3 finalizer of
 * (i + det_drop_seed) > U32_MAX * ratio ? x[i] / (1 - ratio) : 0; 0 < ratio < 1. */
int bh_dropout_inplace(bh_ctx *ctx, float *x, uint64_t n, float ratio, uint32_t det_drop_seed);
/* Softmax over channels per pixel (test/rtc/softmax.cucl). */
int bh_softmax_chans(bh_ctx *ctx, const float *in, float *prob, uint32_t B, uint32_t C, uint32_t H, uint32_t W);
/* Channel-slab copy between NCHW tensors of equal H*W = HW: out[img][oc0 + c] =
 * in[img][ic0 + c] for c < nc. Concat (test/rtc/copy.cucl, ocix) and Split
 * (test/rtc/split_copy.cucl, icix). */
int bh_chan_copy(bh_ctx *ctx, const float *in, float *out, uint32_t B, uint32_t HW, uint32_t in_c, uint32_t ic0,
                 uint32_t out_c, uint32_t oc0, uint32_t nc);

/* Beyond the reference's rtc_fwd (it rejects these), for resnet nets:
 * per-channel affine out = in * scale[c] + shift[c] (+ReLU) -- inference BatchNorm
 * and Scale folded -- over B x C x HW; and Caffe Eltwise of two equal-size tensors,
 * op 0 PROD, 1 SUM, 2 MAX (+ReLU). */
int bh_chan_affine(bh_ctx *ctx, const float *in, float *out, const float *scale, const float *shift, uint32_t B,
                   uint32_t C, uint32_t HW, int relu);
int bh_eltwise(bh_ctx *ctx, const float *a, const float *b, float *out, uint64_t n, int op, int relu);

/* ---- generic device functions through hiprtc: what rtc_compute_t::compile / run do for every
 *      function name the backend does not intercept (the reference JIT-compiles all CUCL with
 *      nvrtc, src/nvrtc_util.cc:216-260, and launches it with cuLaunchKernel, :355-385). src is
 *      the whole program (the caller prepends its CUCL prelude, as nvrtc_compute_t::compile
 *      prepends cu_base_decls); names are the functions to look up (a missing one fails the
 *      compile, src/nvrtc_util.cc check_runnable); opts: extra hiprtc options, space separated
 *      (may be NULL). log (may be NULL) receives the compiler log. ----------------------------- */
/* compile only, no device needed (code_bytes may be NULL) */
int bh_jit_build(const char *src, const char *opts, char *log, size_t loglen, size_t *code_bytes);
int bh_jit_compile(bh_ctx *ctx, const char *src, const char *const *names, int n, const char *opts, int *module_id,
                   char *log, size_t loglen);
/* 1-D launch, blks x tpb; args[i] points at the i-th kernel argument's value (a device pointer
 * variable for a buffer, the value itself for a by-value scalar or struct) -- the reference's
 * arg marshalling (src/nvrtc_util.cc:337-347). An event pair armed by bh_time_next_call is
 * recorded on this launch. */
int bh_jit_launch(bh_ctx *ctx, int module_id, const char *name, void **args, uint32_t blks, uint32_t tpb);
int bh_jit_release(bh_ctx *ctx, int module_id);

/* Name of the kernel variant bh_conv2d_fwd_nchw / bh_sgemm_kmajor would run
 * for a shape (op==0: sgemm with dims[0..2] = M,N,K; op==1: conv with
 * dims[0..10] = B,IC,H,W,OC,KY,KX,sy,sx,py,px). */
int bh_variant_name(int op, const uint32_t *dims, char *buf, size_t buflen);
/* The same, under ctx's bh_tune_set / bh_tune_set_policy overrides: the variant a call on ctx
 * runs now. ops-prof names each tune's run by it -- the role of the generated function name
 * (prc_ret.op->get_func_name(), src/rtc_prof.cc:312) its per-function tolerances key on. */
int bh_variant_name_ctx(bh_ctx *ctx, int op, const uint32_t *dims, char *buf, size_t buflen);

/* ---- tuning (the backend's counterpart of Boda's op_tune sweeps and wisdom,
 *      src/cnn_op.H:10-31, src/op-tuner.cc). Kernel choice per exact shape comes
 *      from, in order: an override set here, the tuning table
 *      (boda-1_amd/tuning/gfx950.tune next to the library, or $BH_TUNE_FILE),
 *      a built-in heuristic. op: 0 = sgemm, 1 = conv. ---------------------- */
/* force tile configuration cfg_index (-1: back to table/heuristic) and K splits
 * for every later call of op on this context: splits 0 = planned, n > 0 = n
 * splits combined in-kernel by each tile's last-arriving block, -n = n splits
 * combined by a separate reduce kernel. Both combines sum in a fixed order.
 * Configuration families reuse splits as their grid mode (direct / Winograd
 * kernels: blocks per CU, whole tiles, + 10 OC tile slowest, + 20 a stream-K
 * grid's cut tiles summed by a second combine kernel). */
int bh_tune_set(bh_ctx *ctx, int op, int cfg_index, int splits);
/* force the output store policy of every later call of op on this context: wt 1 = the outputs
 * are written through (sc1) during the kernel instead of left dirty in L2 for the next kernel
 * boundary to write back; 0 = write-back; -1 = back to the table's / heuristic's choice
 * (tuning tables carry it as " wt=1"). Results are bit-identical either way. */
int bh_tune_set_policy(bh_ctx *ctx, int op, int wt);
/* name of tile configuration cfg_index; BH_UNSUP past the last one */
int bh_tune_cfg_name(int op, int cfg_index, char *buf, size_t buflen);

#ifdef __cplusplus
}
#endif

#endif /* BODA_HIP_H */
