// Host-side launch API of the HIP kernels (plain pointers + hipStream_t; no torch types here, so the
// kernel translation units compile without the PyTorch headers).  bindings.cpp adapts torch tensors.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int kMaxTaps = 49;   // up to 7x7 (ResNet stem)

// Convolution geometry shared by the forward / data-gradient / weight-gradient kernels.
// Inputs and outputs may be split into up to 8 channel GROUPS, each its own NHWC tensor with the
// same padded width: the logical input is the channel-concat of Gi tensors of Cgi channels (UNet's
// torch.cat is never materialised) and the logical output is Go tensors of Cgo channels (Cgo_l of
// them real): horizontally fused sibling convs write each branch's activation straight into its own
// tensor, and the data-gradient of such a fused conv reads the branches' gradients in place.
// Forward:    input pixel of output (oh, ow) for tap t = (oh*stride + dy[t], ow*stride + dx[t]).
// Transposed: input pixel = ((oh + dy[t]) / stride, (ow + dx[t]) / stride) when divisible.
constexpr int kMaxGroups = 8;
struct ConvGeom {
  int N, IH, IW;
  int Gi, Cgi;          // input: Gi tensors [N, IH, IW, Cgi]; Cip = Gi*Cgi
  int OH, OW;
  int Go, Cgo, Cgo_l;   // output: Go tensors [N, OH, OW, Cgo]; GEMM rows = Go*Cgo
  int T, Kp;            // taps, packed K (multiple of 32, >= T*Cip)
  int stride;
  int dy[kMaxTaps], dx[kMaxTaps];
};

struct ConvArgs {
  const uint16_t* x[kMaxGroups];
  uint16_t* y[kMaxGroups];
  const uint16_t* w;    // packed [conv_rows_alloc(Go*Cgo)][Kp]
  const float* bias;    // nullable, [Cgo_l] (Go == 1 only)
  float* stat_part;     // nullable, [conv_stat_blocks][2][Go*Cgo]
  // BN-backward epilogue (data-gradient of a stride-1 conv whose input is the output z of a BatchNorm
  // (+ReLU) read by no other op; Go == 1): the stored output IS dL/dz, and stat_part receives
  // (sum g, sum g*(y - mean)) with g = dz * relu'(y*scale + shift) -- the BN backward's channel partials.
  const uint16_t* bn_y;  // nullable: that BN's input y, [N, OH, OW, Cgo]
  const float* bn_coef;  // [3][Cgo]: scale, shift, mean
  int bn_relu;
  // Deferred-BN input prologue (forward / weight-gradient of a conv whose input group i is the output
  // of a training- or eval-mode BatchNorm(+ReLU) that was never materialised): xc[i] = that BN's
  // [4][Cgi] stats (scale row 0, shift row 1) or nullptr; bit i of xrelu = the BN's ReLU.
  const float* xc[kMaxGroups];
  unsigned xrelu;
  // accumulate: y += conv(x) (the stored bf16 output is read, added in fp32 and re-rounded -- exactly a
  // separate bf16 add); data-gradients of sibling launches that read the same input.  No BN epilogue.
  int accum;
  // Deferred BN-BACKWARD prologue (data-gradient launches on the halo kernel; the mirror of xc): input
  // group i holds dL/dz of a training BatchNorm(+ReLU) whose input y_i is this conv's forward output and
  // whose data-gradient dL/dy was never written.  Staging rebuilds it, bit-identical to bn_act_bwd_apply:
  // dy = k1 * (relu ? [scale*y + shift > 0] : 1) * dz + k2 * y + k3 (bwd8 in common.h).
  // gy[i]: that y (nullptr: the group is a plain gradient); gs[i]: its stats [4][Cgi] (scale, shift rows);
  // gk[i]: its backward coef [3][Cgi]; bit i of grelu: its ReLU.
  const uint16_t* gy[kMaxGroups];
  const float* gs[kMaxGroups];
  const float* gk[kMaxGroups];
  unsigned grelu;
  ConvGeom g;
};

// weight-gradient operands: dY groups, x groups and the x groups' deferred-BN prologue (ConvArgs::xc)
struct WgradPtrs {
  const uint16_t* dy[kMaxGroups];
  const uint16_t* x[kMaxGroups];
  const float* xc[kMaxGroups];
  unsigned xrelu;
  // deferred BN-backward prologue of the dY groups (see ConvArgs::gy; halo weight-gradient only)
  const uint16_t* gy[kMaxGroups];
  const float* gs[kMaxGroups];
  const float* gk[kMaxGroups];
  unsigned grelu;
};

// conv_wgrad_gemm.hip: LDS-tiled weight-gradient GEMM (LDS-DMA staging, transposed fragment reads)
bool conv_wgrad_gemm_ok(const ConvGeom& g, bool trans);
int conv_wgrad_gemm_replicas(const ConvGeom& g, bool pro = false);
int conv_wgrad_gemm(const WgradPtrs& P, float* dw, const ConvGeom& g, bool prologue, hipStream_t s);
void conv_wgrad_gemm_set(int mode);   // 0 off, 1 auto (planner), 2 every eligible conv
int conv_wgrad_gemm_mode();
void conv_wgrad_gemm_force_cfg(int cfg);
int conv_wgrad_gemm_num_cfgs();

// conv.hip
int conv_pick_mi(int rows);
int conv_rows_alloc(int rows);
void conv_set_halo(int on);
void conv_set_halo_split(int mode);   // 0 never, 1 occupancy-preserving (default), 2 wherever it fits
void conv_set_phase(int on);   // phase-decomposed strided TRANS convs (default on; env MSP_CONV_PHASE=0 off)
// bwd: the launch carries a deferred BN-backward prologue (ConvArgs::gy): no PIPE variant, larger table
bool conv_uses_halo(const ConvGeom& g, bool trans, bool bwd = false);
// trans: conv_igemm's flag; bne: a data-gradient launch with the BN-backward epilogue (conv_fwd_bn)
long conv_stat_blocks(const ConvGeom& g, bool trans = false, bool bwd = false, bool bne = false);
// whether conv_wgrad runs the halo weight-gradient kernel (the only one with the BN-backward prologue)
bool conv_wgrad_uses_halo(const ConvGeom& g, bool trans);
// returns 0, or an error code (conv_error_string) -- the bindings raise it as a Python error
int conv_igemm(const ConvArgs& a, bool trans, hipStream_t s);
const char* conv_error_string(int rc);

// conv_gemm.hip: LDS-tiled implicit GEMM (32x32x16 MFMA, LDS-DMA staging) for >= 64-channel inputs
bool conv_gemm_ok(const ConvGeom& g, bool trans);
long conv_gemm_stat_blocks(const ConvGeom& g);
int conv_gemm(const ConvArgs& a, hipStream_t s);
// one phase of a phase-decomposed strided data-gradient on the GEMM kernel (0), or 1: not eligible (gather)
int conv_gemm_phase(const ConvArgs& a, const int* tA, int KW, int s_, int py, int px, int OHf, int OWf,
                    hipStream_t s);
void conv_gemm_set(int on);
void conv_gemm_force_cfg(int cfg);   // tests / A-B: one tile configuration for every launch (-1: planner)
int conv_gemm_num_cfgs();
// dw: fp32 [Go*Cgo][T*Cip] (overwritten)
int conv_plan_selfcheck(int verbose);   // host-only launch-planner invariants (sanitizer harness)
int conv_wgrad_replicas(const ConvGeom& g, bool trans, bool bwd = false, bool pro = false);   // bwd: see conv_wgrad
// xc / xrelu: the deferred-BN prologue of the x groups (see ConvArgs; xc may be nullptr)
// gy/gs/gk/grelu: the deferred BN-backward prologue of the dY groups (nullable; halo kernel only)
int conv_wgrad(const uint16_t* const* dy, const uint16_t* const* x, float* dw, const ConvGeom& g, bool trans,
               const float* const* xc, unsigned xrelu, hipStream_t s, const uint16_t* const* gy = nullptr,
               const float* const* gs = nullptr, const float* const* gk = nullptr, unsigned grelu = 0);
// dst[row][(t_base + t)*Cpk + c_base + c] = src[row*s_row + c*s_ch + t], row < nrow, c < nch, t < T
void pack_weight(const float* src, uint16_t* dst, int nrow, int nch, int T, int Cpk, int Kp, int t_base,
                 int c_base, long s_row, long s_ch, hipStream_t s);
// jobs: int64 [njobs][12] = {src, dst, nrow, nch, T, Cpk, Kp, t_base, c_base, s_row, s_ch, nelem};
// prefix: int32 [njobs] first block of each job (job j owns ceil(nelem/pack_per_block()) blocks)
void pack_batch(const int64_t* jobs, const int* prefix, int njobs, int total_blocks, hipStream_t s);
int pack_per_block();
// dst[row*s_row + c*s_ch + t] (+)= src[row*Ktot + (t_base + t)*Cpk + c_base + c]
void unpack_wgrad(const float* src, float* dst, int nrow, int nch, int T, int Cpk, int Ktot, int t_base, int c_base,
                  long s_row, long s_ch, bool accumulate, int nrep, long rep_stride, hipStream_t s);

// bn.hip  (P = number of pixels, Cp = padded channels; partial buffers are [nblk][2][Cp] fp32)
constexpr int kMaxSumInputs = 8;
constexpr int kTailMax = 6;           // branch-last BNs summed by a DUCK tail (bn_tail_*)
constexpr int kTailMaxCp = 512;       // LDS coefficient tables of the tail passes
long bn_partial_blocks(long P, int Cp);
long bn_tail_blocks(long P, int Cp);
void bn_tail_partial(const uint16_t* dz, const uint16_t* ys, const float* ostats, const float* ocoef, int orelu, int k,
                     const uint16_t* const* y, const float* const* st, unsigned relu, float* part, long P, int Cp,
                     hipStream_t s);
void bn_tail_apply(const uint16_t* dz, const uint16_t* ys, const float* ostats, const float* ocoef, int orelu, int k,
                   const uint16_t* const* y, const float* const* st, const float* const* coef, unsigned relu,
                   uint16_t* const* dy, long P, int Cp, hipStream_t s, uint16_t* g = nullptr);
// (dy[i] nullptr: branch i's data-gradient is deferred to its producer, which rebuilds it from g = out_bn's
// data-gradient, written when g != nullptr)
// coefs[i] (nullable array / entries): deferred-BN prologue of input i (stats rows, ld = Cp), bit i of
// relu_mask its ReLU -- the branch sums that feed a BN read the branches' pre-BN tensors directly.
void sum_stats(const uint16_t* const* inputs, const float* const* coefs, unsigned relu_mask, int k, uint16_t* out,
               float* part, long P, int Cp, hipStream_t s);
// Channel reductions of [nblk][2][width] partials (columns col_off .. col_off+Cp) into an fp64
// workspace tmp[S][2*Cp], S = bn_reduce_splits(nblk); the finalize kernels sum the S rows themselves.
// bn_collapse sums them into out[2*Cp] (fp64) -- the SyncBN path all-reduces that buffer (S = 1).
int bn_reduce_splits(long nblk);
void bn_reduce_partials(const float* part, long nblk, int width, int col_off, int Cp, double* tmp, hipStream_t s);
void bn_collapse(const double* tmp, int S, int Cp, double* out, hipStream_t s);
void bn_finalize(const double* tmp, int S, int C, int Cp, float count, const float* gamma, const float* beta,
                 float* running_mean, float* running_var, float momentum, float eps, int training,
                 float* scale, float* shift, float* mean, float* invstd, hipStream_t s);
int bn_rf_chunks(int Cp);
void bn_reduce_finalize(const float* part, long nblk, int width, int col_off, int C, int Cp, double* tmp,
                        unsigned* cnt, float count, const float* gamma, const float* beta, float* running_mean,
                        float* running_var, float momentum, float eps, float* scale, float* shift, float* mean,
                        float* invstd, hipStream_t s);
void bn_reduce_bwd_finalize(const float* part, long nblk, int C, int Cp, double* tmp, unsigned* cnt, float count,
                            const float* scale, const float* invstd, const float* mean, float* dgamma, float* dbeta,
                            float* coef, float pscale, hipStream_t s);
void bn_act_apply(const uint16_t* y, const float* scale, const float* shift, uint16_t* z, long P, int Cp,
                  int relu, hipStream_t s);
// z = relu(act_a(sa*y + ba) + (sb ? act_b(sb*x + bb) : x)): the ResNet block tail (bitwise the apply + add_act chain)
void bn_add_act(const uint16_t* y, const float* sa, const float* ba, int relu_a, const uint16_t* x, const float* sb,
                const float* bb, int relu_b, uint16_t* z, long P, int Cp, int relu, hipStream_t s);
void bn_act_bwd_partial(const uint16_t* dz, const uint16_t* y, const float* scale, const float* shift,
                        const float* mean, float* part, long P, int Cp, int relu, hipStream_t s);
void bn_bwd_finalize(const double* tmp, int S, int C, int Cp, float count, const float* scale,
                     const float* invstd, const float* mean, float* dgamma, float* dbeta,
                     float* coef, float pscale, hipStream_t s);
void bn_act_bwd_apply(const uint16_t* dz, const uint16_t* y, const float* scale, const float* shift,
                      const float* coef, uint16_t* dy, long P, int Cp, int relu, hipStream_t s);
// + the backward partials of a second BN (scale2 / shift2 / mean2, input y2) whose output is a summand of y: dy is
// that BN's incoming gradient (bn_act_bwd_partial's rows and grid, part [bn_partial_blocks][2][Cp])
void bn_act_bwd_apply_part(const uint16_t* dz, const uint16_t* y, const float* scale, const float* shift,
                           const float* coef, uint16_t* dy, const uint16_t* y2, const float* scale2,
                           const float* shift2, const float* mean2, int relu2, float* part, long P, int Cp, int relu,
                           hipStream_t s);

// elementwise.hip
void nchw_to_nhwc(const float* x, uint16_t* y, int N, int C, int H, int W, int Cp, hipStream_t s);
void nhwc_to_nchw(const uint16_t* x, float* y, int N, int C, int H, int W, int Cp, hipStream_t s);
// lc / sc (nullable): deferred-BN prologues of low / skip (stats rows, ld = Cp)
void up2_add(const uint16_t* low, const uint16_t* skip, uint16_t* out, int N, int h, int w, int Cp,
             const float* lc, int lrelu, const float* sc, int srelu, hipStream_t s);
void pool2_sum(const uint16_t* g, uint16_t* out, int N, int h, int w, int Cp, hipStream_t s);
// coefs (nullable): deferred-BN prologue per input (ld = Cp, the channel width of every input)
void relu6(const uint16_t* x, uint16_t* y, long n_elem, hipStream_t s);   // min(max(x, 0), 6)
// 8-channel pixels: out = [relu(s*x + h) (C ch), (s*x + h > 0) (C ch), 0 ...], C <= 4; stats [4][8] rows scale, shift
void bn_aug_mask(const uint16_t* x, const float* stats, uint16_t* out, long npix, int C, hipStream_t s);
void relu6_bwd(const uint16_t* dy, const uint16_t* y, uint16_t* dx, long n_elem, hipStream_t s);
void add_n(const uint16_t* const* inputs, const float* const* coefs, unsigned relu_mask, int k, uint16_t* out,
           long n_elem, int Cp, hipStream_t s);
void scale_f32(float* x, const float* scalar, float mult, long n, hipStream_t s);

// pool.hip  (NHWC bf16; idx = one byte per element = winning tap r*k+c)
void maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* idx, int N, int IH, int IW, int OH, int OW, int Cp, int k,
                 int s, int p, hipStream_t st);
void maxpool_bwd(const uint16_t* dy, const uint8_t* idx, uint16_t* dx, int N, int IH, int IW, int OH, int OW, int Cp,
                 int k, int s, int p, hipStream_t st);
void up2_cat(const uint16_t* low, const uint16_t* skip, uint16_t* out, int N, int h, int w, int Cl, int Cpl, int Cs,
             int Cps, int Cpo, hipStream_t st);
void up2_cat_bwd(const uint16_t* g, uint16_t* dlow, uint16_t* dskip, int N, int h, int w, int Cl, int Cpl, int Cs,
                 int Cps, int Cpo, hipStream_t st);
void add_act(const uint16_t* a, const uint16_t* b, uint16_t* z, long n_elem, int relu, hipStream_t st);
void relu_bwd(const uint16_t* dz, const uint16_t* z, uint16_t* g, long n_elem, hipStream_t st);

// augment.hip  (HBM-resident uint8 dataset; see augment.hip for the per-sample parameter layout)
constexpr int kAugIParams = 14;
void aug_geometry(const uint8_t* images, const uint8_t* masks, const int64_t* meta, const int* ip, float* work,
                  int64_t* mask_out, int B, int CH, int CW, hipStream_t s);
int aug_gray_scratch_doubles(int B);   // fp64 partials aug_gray_mean needs
void aug_gray_mean(const float* work, float* mean, double* part, int B, int HW, hipStream_t s);
void aug_color(float* work, const int* ip, const float* fp, const float* mean, int B, int HW, int stage,
               hipStream_t s);
void aug_finalize(const float* work, const int* ip, float* out, int B, int HW, const float* mean3, const float* std3,
                  hipStream_t s);

// loss.hip  (logits NCHW fp32 [N, C, HW]; targets int64 [N, HW])
long ce_blocks(long P);
void ce_fwd_bwd(const float* logits, const int64_t* target, const float* weight, float* grad,
                float* pix_loss, float* part, int N, int C, long HW, int ignore_index, hipStream_t s);
void kd_kl_fwd_bwd(const float* s_logits, const float* t_logits, float* grad, float* part, int N, int C,
                   long HW, float T, hipStream_t s);
// OHEM on the device (no host sync): bpart fp32 [ce_blocks(P)][3], state uint32 [ohem_state_words()],
// hist uint32 [256], loss fp32 [1]; backward scales the CE gradient in place by g * w(pixel)
int ohem_state_words();
void ohem_select(const float* pix_loss, const int64_t* target, long P, float thr, int ignore_index, float* bpart,
                 unsigned* state, unsigned* hist, float* loss, hipStream_t s);
void ohem_backward(float* grad, const float* pix_loss, const unsigned* state, const float* gup, int N, int C, long HW,
                   hipStream_t s);
// part[ce_blocks(n)] = partial sums of (s - t)^2; grad = 2 (s - t) / n
void mse_fwd_bwd(const float* s_, const float* t, float* grad, float* part, long n, hipStream_t s);
// binary logits / targets fp32 [N, HW]: part [N][bce_dice_splits(HW)][4]; coef [N][2]; gup device scalar
int bce_dice_splits(long HW);
void bce_dice_stats(const float* x, const float* t, float* part, int N, long HW, hipStream_t s);
void bce_dice_grad(const float* x, const float* t, const float* coef, const float* gup, float* grad, int N, long HW,
                   float bw, float dw, hipStream_t s);

// optim.hip  (flat fp32 buffers; hyper = device fp32 array, see optim.hip for the layout)
void adam_step(float* p, const float* g, float* m, float* v, const float* hyper, long n, int adamw,
               const float* amp, hipStream_t s);
void sgd_step(float* p, const float* g, float* buf, const float* hyper, long n, const float* amp, hipStream_t s);
void amp_check(const float* g, long n, float* amp, hipStream_t s);
void amp_update(float* amp, float growth, float backoff, int interval, hipStream_t s);
void ema_update(float* ema, const float* model, const float* hyper, long n, hipStream_t s);

// metrics.hip
void confmat_update(const float* logits, const int64_t* target, int64_t* confmat, int N, int C, long HW,
                    int ignore_index, hipStream_t s);
void bilinear_resize(const float* x, float* y, long NC, int IH, int IW, int OH, int OW, int align_corners,
                     hipStream_t s);
void colorize(const float* logits, const uint8_t* lut, uint8_t* rgb, int N, int C, long HW, hipStream_t s);

// decoder.hip: smp decoder-hub ops (bilinear resize, GroupNorm, adaptive pooling, depthwise conv)
void resize_bilinear_fwd(const uint16_t* x, uint16_t* y, int N, int IH, int IW, int OH, int OW, int Cp, float sh,
                         float sw, int align, int accum, hipStream_t s);
void resize_bilinear_bwd(const uint16_t* dy, uint16_t* dx, int N, int IH, int IW, int OH, int OW, int Cp, float sh,
                         float sw, int align, hipStream_t s);
int nc_sums_blocks(long HW, int Cp);
void nc_sums(const uint16_t* x, const uint16_t* dz, const float* tab, int relu, int N, long HW, int Cp, float* part,
             int nblk, hipStream_t s);
void gn_finalize(const float* part, int nblk, int N, int C, int Cp, int G, float eps, const float* gamma,
                 const float* beta, long HW, float* tab, hipStream_t s);
void gn_bwd_finalize(const float* part, int nblk, int N, int C, int Cp, int G, const float* gamma, const float* tab,
                     long HW, float* dgamma, float* dbeta, float* coef, hipStream_t s);
void affine_nc(const uint16_t* x, const float* tab, int rows, uint16_t* z, int N, long HW, int Cp, int relu,
               hipStream_t s);
void affine_nc_bwd(const uint16_t* dz, const uint16_t* x, const float* tab, const float* coef, uint16_t* dx, int N,
                   long HW, int Cp, int relu, hipStream_t s);
void adaptive_avgpool_fwd(const uint16_t* x, uint16_t* y, int N, int H, int W, int OH, int OW, int Cp, hipStream_t s);
void adaptive_avgpool_bwd(const uint16_t* dy, uint16_t* dx, int N, int H, int W, int OH, int OW, int Cp,
                          hipStream_t s);
void dwconv_fwd(const uint16_t* x, const float* w, const float* bias, uint16_t* y, int N, int H, int W, int Cp, int T,
                const int* dy, const int* dx, hipStream_t s);
int dwconv_wgrad_blocks(long P, int Cp);
int dwconv_wgrad(const uint16_t* x, const uint16_t* dyv, float* part, int nblk, int N, int H, int W, int Cp, int T,
                 const int* dy, const int* dx, hipStream_t s);
void colsum(const float* part, int nrow, int ncol, float* out, int accum, hipStream_t s);

// comm.hip: one-shot intra-node all-reduce over IPC-mapped peer buffers (SyncBN statistic exchanges)
constexpr int kCommMaxRanks = 16;
constexpr long kCommDataOff = 4096;       // flags first, then data[2][world][cap] fp64
constexpr int kCommHandleBytes = 64;
struct CommPeers {
  char* buf[kCommMaxRanks];               // every rank's exchange buffer, mapped in this process
};
long comm_buffer_bytes(long cap, int world);
int comm_alloc(long bytes, void** ptr, void* handle64);
int comm_open(const void* handle64, void** ptr);
void comm_close(void* ptr);
void comm_free(void* ptr);
void oneshot_allreduce(const double* in, double* out, long n, const CommPeers& peers, int rank, int world, long cap,
                       unsigned long long* epoch, int nstate, int* err, long long timeout, hipStream_t s);

// conv_bwd.hip: fused data- + weight-gradient of a narrow stride-1 conv (one staging of dY and x per tile).
// Geometry = the FORWARD conv (Gi = Go = 1, Cgi, Cgo <= 32, symmetric taps).  dY = bwd(dz, gy) when gy is set
// (deferred BN-backward, gs/gk/grelu as ConvArgs::gy), else dz; x = relu?(xc scale/shift prologue) when xc is
// set.  dxo <- dL/dx [N,H,W,Cgi]; bn_y/bn_coef/bn_relu/stat_part: the BN-backward partials epilogue (ConvArgs).
// dw <- [conv_bwd_fused_blocks][Cgo][T*Cgi] fp32 slabs (summed by unpack_wgrad).  wd: the packed data-gradient
// weights (ConvPlan.pack_dgrad), Kp = their row pitch.
constexpr int kFusedBwdGrid = 256;   // persistent grid: one (staging + compute waves) block per CU
struct FusedBwdArgs {
  const uint16_t* dz;
  const uint16_t* gy;
  const float* gs;
  const float* gk;
  int grelu;
  // Go == 2: a second output group (the ResidualBlock's 1x1 shortcut riding in the 3x3's launch) with its
  // own dY (rebuilt from its own deferred BN gradient when gy2 != nullptr) at the single forward tap t1
  int Go, t1;
  const uint16_t* dz2;
  const uint16_t* gy2;
  const float* gs2;
  const float* gk2;
  int grelu2;
  const uint16_t* x;
  const float* xc;
  int xrelu;
  const uint16_t* wd;
  int Kp;
  uint16_t* dxo;
  const uint16_t* bn_y;
  const float* bn_coef;
  int bn_relu;
  float* stat_part;
  float* dw;
  int N, H, W, Ci, Co, T;
  int dy[9], dx[9];
  // forward mode (conv_fwd_fused): per-output-channel bias (nullable) over the Co_l logical channels;
  // opitch = the output tensors' channel pitch.  co_split > 0: two output groups (the ResidualBlock's 3x3 +
  // 1x1 pair, stacked rows): rows >= co_split go to dxo2 at channel row - co_split.
  const float* bias;
  int Co_l;
  uint16_t* dxo2;
  int co_split, opitch;
  // backward: dx += this launch's data-gradient (the DUCK first convs' sibling launches sum into one dL/dx;
  // a BN epilogue then sees the summed values)
  int accum;
  // data-gradient K-unit order (set by conv_bwd_fused): unit index, or -1 for a zero-weight padding unit.  Paired k-groups (0/1, 2/3) share a ds_read_b128 lane group: units paired with
  // equal slot offsets mod 16 read conflict-free.
  short uperm[96];
};
struct FusedBwdGeom {
  int TH, TW, tw_shift, HH, HWD, ey0, ex0, tiles_y, tiles_x, ntiles;
  int py, px, KS, nj, cw, cb;   // cw: compute waves (4 or 8), cb: 16-channel blocks (2 or 3) (conv_bwd.hip)
  float inv_c8y, inv_c8x, inv_hwd;   // fp32 reciprocals (fdiv) of the staging index math
};
bool conv_bwd_fused_plan(const ConvGeom& g, FusedBwdGeom& fg);
int conv_bwd_fused_blocks(const ConvGeom& g);   // 0: not eligible
int conv_bwd_fused(const FusedBwdArgs& a, const ConvGeom& g, hipStream_t s);
// The same persistent staging / compute-wave kernel as a FORWARD conv (stride 1, one input and one output
// group of <= 32 channels each, T >= 2: the 17-channel level's 3x3 / dilated / 1x7 convs): x staged through
// the deferred-BN prologue, y + its BN statistics (per-block partial rows, conv_stat_blocks) in the epilogue.
bool conv_fwd_fused_ok(const ConvGeom& g);
long conv_fwd_fused_blocks(const ConvGeom& g);   // its stat partial rows (persistent grid)
void conv_set_fwd_fused(int on);                   // A/B and tests (default: env MSP_CONV_FWD_FUSED, on)
int conv_fwd_fused(const ConvArgs& a, hipStream_t s);

// attention.hip: batched bf16 GEMM C[b] = op(A[b]) . op(B[b]) (fp32 accumulation, bf16 / fp32 out) and the
// whole-map softmax (+ backward) of MAnet's position-attention block
int batched_gemm(const uint16_t* A, const uint16_t* B, void* C, bool out_bf16, int batch, int M, int N, int K, int lda,
                 int ldb, int ldc, long sa, long sb, long sc, bool transA, bool transB, hipStream_t s);
void softmax_all(const float* S, uint16_t* P, int batch, long n, hipStream_t s);
void softmax_all_bwd(const uint16_t* P, const float* dP, uint16_t* dS, int batch, long n, hipStream_t s);

// gconv.hip: grouped convolution (ResNeXt grouped 3x3), NHWC bf16, fp32 weights repacked [T][C][CG]
int gconv_fwd(const uint16_t* x, const float* w, uint16_t* y, int N, int IH, int IW, int OH, int OW, int C, int CG,
              int stride, int T, const int* dyv, const int* dxv, hipStream_t s);
int gconv_dgrad(const uint16_t* dy, const float* w, uint16_t* dx, int N, int IH, int IW, int OH, int OW, int C, int CG,
                int stride, int T, const int* dyv, const int* dxv, hipStream_t s);
int gconv_wgrad_slices(long P, int C, int CG, int T);
// MFMA weight-gradient: part [nslice][C/16][9*KW/16][16][16] (colsum over slices; block diagonal on the host)
int gconv_wgrad_mfma_slices(long P, int C);
int gconv_wgrad_mfma(const uint16_t* x, const uint16_t* dy, float* part, int nslice, int N, int IH, int IW, int OH,
                     int OW, int C, int KW, int stride, int T, const int* dyv, const int* dxv, hipStream_t s);
// MFMA forward / data-gradient (trans): wpk bf16 [C/16][ceil(9*KW/32)][64][8], KW = max(16, CG); 3x3 only
int gconv_mfma(const uint16_t* x, const uint16_t* wpk, uint16_t* y, int N, int IH, int IW, int OH, int OW, int C,
               int KW, int stride, bool trans, int T, const int* dyv, const int* dxv, hipStream_t s);
// part [nslice][T * C/8 * max(1, CG/8)][64] fp32 (summed over slices by colsum)
int gconv_wgrad(const uint16_t* x, const uint16_t* dy, float* part, int nslice, int N, int IH, int IW, int OH, int OW,
                int C, int CG, int stride, int T, const int* dyv, const int* dxv, hipStream_t s);
