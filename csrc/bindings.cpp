// PyTorch binding of the MI355X kernels (module `medical_segmentation_pytorch_amd._C`).
// Thin adapters only: shape/dtype/device checks, then the plain launchers in launchers.h on the
// current HIP stream (so everything composes with torch streams and hipGraph capture).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <algorithm>
#include <vector>

#include "launchers.h"

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda() && (t).is_contiguous(), #t " must be a contiguous GPU tensor")
#define CHECK_BF16(t) CHECK_DEV(t); TORCH_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bf16")
#define CHECK_F32(t) CHECK_DEV(t); TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be fp32")
#define CHECK_I64(t) CHECK_DEV(t); TORCH_CHECK((t).scalar_type() == at::kLong, #t " must be int64")

inline uint16_t* bf(const at::Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }
inline float* f32(const at::Tensor& t) { return t.data_ptr<float>(); }
inline const float* f32_opt(const c10::optional<at::Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  CHECK_F32(*t);
  return t->data_ptr<float>();
}
inline float* f32_opt_mut(const c10::optional<at::Tensor>& t) { return const_cast<float*>(f32_opt(t)); }

using OptTensors = std::vector<c10::optional<at::Tensor>>;

// deferred-BN prologue coefficient rows: entry i = that input's BN stats [4][ld] fp32 (or None)
void fill_coefs(const OptTensors& cs, int n, const std::vector<int64_t>& ld, const float** out) {
  TORCH_CHECK(cs.empty() || (int)cs.size() == n, "one prologue entry per input");
  for (int i = 0; i < n; ++i) {
    out[i] = nullptr;
    if (cs.empty() || !cs[i].has_value() || !cs[i]->defined()) continue;
    CHECK_F32(*cs[i]);
    TORCH_CHECK(cs[i]->numel() >= 2 * ld[i], "prologue coefficients must hold [scale; shift] rows of the input width");
    out[i] = cs[i]->data_ptr<float>();
  }
}

// deferred BN-backward prologue of the data-gradient groups (ConvArgs::gy): per group the BN input y (bf16,
// the group's shape), its stats [4][C] and backward coef [3][C] (fp32), or None for a plain gradient group
bool fill_bwd(const OptTensors& ys, const OptTensors& ss, const OptTensors& ks, int n, int64_t numel, int64_t C,
              const uint16_t** gy, const float** gs, const float** gk) {
  TORCH_CHECK(ys.empty() || ((int)ys.size() == n && (int)ss.size() == n && (int)ks.size() == n),
              "BN-backward prologue: one (y, stats, coef) entry per gradient group");
  bool any = false;
  for (int i = 0; i < n; ++i) {
    gy[i] = nullptr; gs[i] = nullptr; gk[i] = nullptr;
    if (ys.empty() || !ys[i].has_value() || !ys[i]->defined()) continue;
    CHECK_BF16(*ys[i]);
    TORCH_CHECK(ys[i]->numel() == numel, "BN-backward prologue: y must have the gradient's shape");
    TORCH_CHECK(ss[i].has_value() && ks[i].has_value(), "BN-backward prologue: stats and coef required");
    CHECK_F32(*ss[i]); CHECK_F32(*ks[i]);
    TORCH_CHECK(ss[i]->numel() >= 2 * C && ks[i]->numel() >= 3 * C, "BN-backward prologue: [4][C] stats, [3][C] coef");
    gy[i] = bf(*ys[i]); gs[i] = ss[i]->data_ptr<float>(); gk[i] = ks[i]->data_ptr<float>();
    any = true;
  }
  return any;
}

ConvGeom make_geom(const std::vector<int64_t>& dims, const std::vector<int64_t>& dy, const std::vector<int64_t>& dx) {
  TORCH_CHECK(dims.size() == 13, "geom dims = [N, IH, IW, Gi, Cgi, OH, OW, Go, Cgo, Cgo_l, T, Kp, stride]");
  ConvGeom g{};
  g.N = dims[0]; g.IH = dims[1]; g.IW = dims[2]; g.Gi = dims[3]; g.Cgi = dims[4];
  g.OH = dims[5]; g.OW = dims[6]; g.Go = dims[7]; g.Cgo = dims[8]; g.Cgo_l = dims[9];
  g.T = dims[10]; g.Kp = dims[11]; g.stride = dims[12];
  TORCH_CHECK(g.T >= 1 && g.T <= kMaxTaps && (int)dy.size() == g.T && (int)dx.size() == g.T, "bad tap table");
  TORCH_CHECK(g.Gi >= 1 && g.Gi <= kMaxGroups && g.Go >= 1 && g.Go <= kMaxGroups, "1..8 channel groups");
  TORCH_CHECK(g.Cgi % 8 == 0 && g.Cgo % 8 == 0, "channel dims must be padded to a multiple of 8");
  TORCH_CHECK(g.Kp % 32 == 0 && g.Kp >= g.T * g.Gi * g.Cgi, "Kp must be a multiple of 32 covering T*Cip");
  TORCH_CHECK(g.Cgo_l <= g.Cgo && g.stride >= 1, "bad output channels / stride");
  for (int i = 0; i < g.T; ++i) { g.dy[i] = dy[i]; g.dx[i] = dx[i]; }
  return g;
}

void conv_fwd(std::vector<at::Tensor> xs, const at::Tensor& wp, std::vector<at::Tensor> ys,
              const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& stat_part,
              std::vector<int64_t> dims, std::vector<int64_t> dy, std::vector<int64_t> dx, bool trans,
              OptTensors xc, int64_t xrelu, bool accumulate, OptTensors gy, OptTensors gs, OptTensors gk,
              int64_t grelu) {
  ConvGeom g = make_geom(dims, dy, dx);
  TORCH_CHECK(!accumulate || !(stat_part.has_value() && stat_part->defined()), "accumulate: no stats epilogue");
  TORCH_CHECK((int)xs.size() == g.Gi && (int)ys.size() == g.Go, "group count mismatch");
  ConvArgs a{};
  for (int i = 0; i < g.Gi; ++i) {
    CHECK_BF16(xs[i]);
    TORCH_CHECK(xs[i].numel() == (int64_t)g.N * g.IH * g.IW * g.Cgi, "x numel mismatch");
    a.x[i] = bf(xs[i]);
  }
  for (int i = 0; i < g.Go; ++i) {
    CHECK_BF16(ys[i]);
    TORCH_CHECK(ys[i].numel() == (int64_t)g.N * g.OH * g.OW * g.Cgo, "y numel mismatch");
    a.y[i] = bf(ys[i]);
  }
  CHECK_BF16(wp);
  TORCH_CHECK(wp.numel() == (int64_t)conv_rows_alloc(g.Go * g.Cgo) * g.Kp, "packed weight numel mismatch");
  if (bias.has_value() && bias->defined()) TORCH_CHECK(g.Go == 1 && bias->numel() == g.Cgo_l, "bias: 1 group only");
  const bool bwd = fill_bwd(gy, gs, gk, g.Gi, (int64_t)g.N * g.IH * g.IW * g.Cgi, g.Cgi, a.gy, a.gs, a.gk);
  a.grelu = (unsigned)grelu;
  if (stat_part.has_value() && stat_part->defined())
    TORCH_CHECK(stat_part->numel() == conv_stat_blocks(g, trans, bwd) * 2 * g.Go * g.Cgo, "stat_part numel mismatch");
  a.w = bf(wp);
  a.bias = f32_opt(bias);
  a.stat_part = f32_opt_mut(stat_part);
  fill_coefs(xc, g.Gi, std::vector<int64_t>(g.Gi, g.Cgi), a.xc);
  a.xrelu = (unsigned)xrelu;
  a.accum = accumulate ? 1 : 0;
  a.g = g;
  const int rc = conv_igemm(a, trans, cur_stream());
  TORCH_CHECK(rc == 0, conv_error_string(rc));
}

// Data-gradient launch with the BN-backward epilogue (see ConvArgs::bn_y): stat_part receives the
// channel partials of the BatchNorm whose output z was this conv's only input.
void conv_fwd_bn(std::vector<at::Tensor> xs, const at::Tensor& wp, std::vector<at::Tensor> ys, const at::Tensor& stat_part,
                 std::vector<int64_t> dims, std::vector<int64_t> dy, std::vector<int64_t> dx, const at::Tensor& bn_y,
                 const at::Tensor& bn_coef, bool relu, OptTensors gy, OptTensors gs, OptTensors gk, int64_t grelu) {
  ConvGeom g = make_geom(dims, dy, dx);
  TORCH_CHECK(g.Go == 1 && (int)ys.size() == 1 && (int)xs.size() == g.Gi, "BN epilogue: one output group");
  ConvArgs a{};
  for (int i = 0; i < g.Gi; ++i) {
    CHECK_BF16(xs[i]);
    TORCH_CHECK(xs[i].numel() == (int64_t)g.N * g.IH * g.IW * g.Cgi, "x numel mismatch");
    a.x[i] = bf(xs[i]);
  }
  CHECK_BF16(ys[0]);
  TORCH_CHECK(ys[0].numel() == (int64_t)g.N * g.OH * g.OW * g.Cgo, "y numel mismatch");
  a.y[0] = bf(ys[0]);
  CHECK_BF16(wp);
  TORCH_CHECK(wp.numel() == (int64_t)conv_rows_alloc(g.Go * g.Cgo) * g.Kp, "packed weight numel mismatch");
  const bool bwd = fill_bwd(gy, gs, gk, g.Gi, (int64_t)g.N * g.IH * g.IW * g.Cgi, g.Cgi, a.gy, a.gs, a.gk);
  a.grelu = (unsigned)grelu;
  CHECK_F32(stat_part);
  TORCH_CHECK(stat_part.numel() == conv_stat_blocks(g, false, bwd, true) * 2 * g.Cgo, "stat_part numel mismatch");
  CHECK_BF16(bn_y);
  TORCH_CHECK(bn_y.numel() == ys[0].numel(), "bn_y must have the data-gradient's shape");
  CHECK_F32(bn_coef);
  TORCH_CHECK(bn_coef.numel() >= 3 * (int64_t)g.Cgo, "bn_coef = [scale; shift; mean] rows of Cgo");
  TORCH_CHECK(g.stride == 1, "BN epilogue: stride-1 data-gradients only");
  a.w = bf(wp);
  a.stat_part = f32(stat_part);
  a.bn_y = bf(bn_y);
  a.bn_coef = f32(bn_coef);
  a.bn_relu = relu ? 1 : 0;
  a.g = g;
  const int rc = conv_igemm(a, false, cur_stream());
  TORCH_CHECK(rc == 0, conv_error_string(rc));
}

void conv_wgrad_t(std::vector<at::Tensor> dys, std::vector<at::Tensor> xs, const at::Tensor& dw,
                  std::vector<int64_t> dims, std::vector<int64_t> dy, std::vector<int64_t> dx, bool trans,
                  OptTensors xc, int64_t xrelu, OptTensors gy, OptTensors gs, OptTensors gk, int64_t grelu) {
  ConvGeom g = make_geom(dims, dy, dx);
  TORCH_CHECK((int)xs.size() == g.Gi && (int)dys.size() == g.Go, "group count mismatch");
  std::vector<const uint16_t*> px, pd;
  for (auto& t : xs) { CHECK_BF16(t); TORCH_CHECK(t.numel() == (int64_t)g.N * g.IH * g.IW * g.Cgi); px.push_back(bf(t)); }
  for (auto& t : dys) { CHECK_BF16(t); TORCH_CHECK(t.numel() == (int64_t)g.N * g.OH * g.OW * g.Cgo); pd.push_back(bf(t)); }
  CHECK_F32(dw);
  const int64_t one = (int64_t)g.Go * g.Cgo * g.T * g.Gi * g.Cgi;
  const uint16_t* gyp[kMaxGroups];
  const float* gsp[kMaxGroups];
  const float* gkp[kMaxGroups];
  const bool bwd = fill_bwd(gy, gs, gk, g.Go, (int64_t)g.N * g.OH * g.OW * g.Cgo, g.Cgo, gyp, gsp, gkp);
  const float* cf[kMaxGroups];
  fill_coefs(xc, g.Gi, std::vector<int64_t>(g.Gi, g.Cgi), cf);
  bool pro = false;
  for (int i = 0; i < g.Gi; ++i) pro |= cf[i] != nullptr;
  TORCH_CHECK(dw.numel() == one * conv_wgrad_replicas(g, trans, bwd, pro), "dw numel mismatch (replicas)");
  TORCH_CHECK(!trans || xc.empty(), "no BN prologue on transposed weight-gradients");
  const int rc = conv_wgrad(pd.data(), px.data(), f32(dw), g, trans, cf, (unsigned)xrelu, cur_stream(), gyp, gsp, gkp,
                            (unsigned)grelu);
  TORCH_CHECK(rc == 0, conv_error_string(rc));
}

int64_t conv_wgrad_replicas_t(std::vector<int64_t> dims, std::vector<int64_t> dy, std::vector<int64_t> dx, bool trans,
                              bool bwd, bool pro) {
  return conv_wgrad_replicas(make_geom(dims, dy, dx), trans, bwd, pro);
}

bool conv_uses_halo_t(std::vector<int64_t> dims, std::vector<int64_t> dy, std::vector<int64_t> dx, bool trans, bool bwd) {
  return conv_uses_halo(make_geom(dims, dy, dx), trans, bwd);
}

bool conv_wgrad_uses_halo_t(std::vector<int64_t> dims, std::vector<int64_t> dy, std::vector<int64_t> dx, bool trans) {
  return conv_wgrad_uses_halo(make_geom(dims, dy, dx), trans);
}

int64_t conv_stat_blocks_t(std::vector<int64_t> dims, std::vector<int64_t> dy, std::vector<int64_t> dx, bool trans,
                           bool bwd, bool bne) {
  return conv_stat_blocks(make_geom(dims, dy, dx), trans, bwd, bne);
}

void pack_weight_t(const at::Tensor& src, const at::Tensor& dst, int64_t nrow, int64_t nch, int64_t T, int64_t Cpk,
                   int64_t Kp, int64_t t_base, int64_t c_base, int64_t s_row, int64_t s_ch) {
  CHECK_F32(src); CHECK_BF16(dst);
  TORCH_CHECK(dst.numel() >= nrow * Kp && (t_base + T - 1) * Cpk + c_base + nch <= Kp, "dst too small");
  TORCH_CHECK(src.numel() >= (nrow - 1) * s_row + (nch - 1) * s_ch + T, "src too small");
  pack_weight(f32(src), bf(dst), nrow, nch, T, Cpk, Kp, t_base, c_base, s_row, s_ch, cur_stream());
}

void unpack_wgrad_t(const at::Tensor& src, const at::Tensor& dst, int64_t nrow, int64_t nch, int64_t T, int64_t Cpk,
                    int64_t Ktot, int64_t t_base, int64_t c_base, int64_t s_row, int64_t s_ch, bool accumulate,
                    int64_t nrep, int64_t rep_stride) {
  CHECK_F32(src);
  TORCH_CHECK(dst.is_cuda() && dst.scalar_type() == at::kFloat, "dst must be fp32 GPU");
  TORCH_CHECK(nrep >= 1 && (nrep == 1 || rep_stride >= nrow * Ktot), "bad replica layout");
  TORCH_CHECK(src.numel() >= (nrep - 1) * rep_stride + nrow * Ktot && (t_base + T - 1) * Cpk + c_base + nch <= Ktot,
              "src too small");
  TORCH_CHECK(dst.numel() >= (nrow - 1) * s_row + (nch - 1) * s_ch + T, "dst too small");
  unpack_wgrad(f32(src), dst.data_ptr<float>(), nrow, nch, T, Cpk, Ktot, t_base, c_base, s_row, s_ch, accumulate,
               (int)nrep, rep_stride, cur_stream());
}

void pack_batch_t(const at::Tensor& jobs, const at::Tensor& prefix, int64_t total_blocks) {
  CHECK_I64(jobs);
  CHECK_DEV(prefix);
  TORCH_CHECK(prefix.scalar_type() == at::kInt && jobs.dim() == 2 && jobs.size(1) == 12 &&
              prefix.numel() == jobs.size(0), "pack_batch: bad job table");
  pack_batch(jobs.data_ptr<int64_t>(), prefix.data_ptr<int>(), (int)jobs.size(0), (int)total_blocks, cur_stream());
}

void sum_stats_t(std::vector<at::Tensor> inputs, const c10::optional<at::Tensor>& out, const at::Tensor& part,
                 int64_t P, int64_t Cp, OptTensors coefs, int64_t relu_mask) {
  TORCH_CHECK(!inputs.empty() && (int)inputs.size() <= kMaxSumInputs, "1..8 inputs");
  TORCH_CHECK(Cp % 8 == 0 && Cp <= 2048, "Cp must be a multiple of 8, <= 2048");
  std::vector<const uint16_t*> ptrs;
  for (auto& t : inputs) { CHECK_BF16(t); TORCH_CHECK(t.numel() == P * Cp, "input numel mismatch"); ptrs.push_back(bf(t)); }
  uint16_t* o = nullptr;
  if (out.has_value() && out->defined()) { CHECK_BF16(*out); TORCH_CHECK(out->numel() == P * Cp); o = bf(*out); }
  CHECK_F32(part);
  TORCH_CHECK(part.numel() == bn_partial_blocks(P, Cp) * 2 * Cp, "part numel mismatch");
  const float* cf[kMaxSumInputs];
  fill_coefs(coefs, (int)ptrs.size(), std::vector<int64_t>(ptrs.size(), Cp), cf);
  for (int i = 0; i < (int)ptrs.size(); ++i) TORCH_CHECK(cf[i] == nullptr || o != nullptr, "prologue needs out");
  sum_stats(ptrs.data(), cf, (unsigned)relu_mask, (int)ptrs.size(), o, f32(part), P, Cp, cur_stream());
}

#define CHECK_F64(t) CHECK_DEV(t); TORCH_CHECK((t).scalar_type() == at::kDouble, #t " must be fp64")

// tmp: fp64 [S, 2*Cp] with S = bn_reduce_splits(nblk)
void bn_reduce_partials_t(const at::Tensor& part, int64_t nblk, int64_t width, int64_t col_off, int64_t Cp,
                          const at::Tensor& tmp) {
  CHECK_F32(part); CHECK_F64(tmp);
  TORCH_CHECK(part.numel() == nblk * 2 * width && col_off + Cp <= width, "partials size mismatch");
  TORCH_CHECK(tmp.numel() == (int64_t)bn_reduce_splits(nblk) * 2 * Cp, "tmp must be [bn_reduce_splits(nblk), 2*Cp]");
  bn_reduce_partials(f32(part), nblk, width, col_off, Cp, tmp.data_ptr<double>(), cur_stream());
}

void bn_collapse_t(const at::Tensor& tmp, int64_t Cp, const at::Tensor& out) {
  CHECK_F64(tmp); CHECK_F64(out);
  TORCH_CHECK(tmp.numel() % (2 * Cp) == 0 && out.numel() == 2 * Cp);
  bn_collapse(tmp.data_ptr<double>(), (int)(tmp.numel() / (2 * Cp)), Cp, out.data_ptr<double>(), cur_stream());
}

void bn_finalize_t(const at::Tensor& tmp, int64_t C, int64_t Cp, double count, const c10::optional<at::Tensor>& gamma,
                   const c10::optional<at::Tensor>& beta, const c10::optional<at::Tensor>& rmean,
                   const c10::optional<at::Tensor>& rvar, double momentum, double eps, bool training,
                   const at::Tensor& stats) {
  CHECK_F64(tmp); CHECK_F32(stats);
  TORCH_CHECK(stats.numel() == 4 * Cp, "stats = [scale, shift, mean, invstd] x Cp");
  TORCH_CHECK(tmp.numel() % (2 * Cp) == 0, "tmp must be [S, 2*Cp]");
  TORCH_CHECK(training || (rmean.has_value() && rvar.has_value()), "eval BN needs running stats");
  float* st = f32(stats);
  bn_finalize(tmp.data_ptr<double>(), (int)(tmp.numel() / (2 * Cp)), C, Cp, (float)count, f32_opt(gamma),
              f32_opt(beta), f32_opt_mut(rmean), f32_opt_mut(rvar), (float)momentum, (float)eps, training ? 1 : 0,
              st, st + Cp, st + 2 * Cp, st + 3 * Cp, cur_stream());
}

void bn_reduce_finalize_t(const at::Tensor& part, int64_t nblk, int64_t width, int64_t col_off, int64_t C, int64_t Cp,
                          const at::Tensor& tmp, const at::Tensor& cnt, double count,
                          const c10::optional<at::Tensor>& gamma, const c10::optional<at::Tensor>& beta,
                          const c10::optional<at::Tensor>& rmean, const c10::optional<at::Tensor>& rvar,
                          double momentum, double eps, const at::Tensor& stats) {
  CHECK_F32(part); CHECK_F64(tmp); CHECK_F32(stats); CHECK_DEV(cnt);
  TORCH_CHECK(cnt.scalar_type() == at::kInt && cnt.numel() >= bn_rf_chunks(Cp), "cnt: int32 >= Cp/32 counters");
  TORCH_CHECK(part.numel() >= nblk * 2 * width && col_off + Cp <= width, "partials too small");
  TORCH_CHECK(tmp.numel() >= (int64_t)bn_reduce_splits(nblk) * 2 * Cp, "tmp too small");
  TORCH_CHECK(stats.numel() == 4 * Cp, "stats = [scale, shift, mean, invstd] x Cp");
  float* st = f32(stats);
  bn_reduce_finalize(f32(part), nblk, width, col_off, C, Cp, tmp.data_ptr<double>(),
                     reinterpret_cast<unsigned*>(cnt.data_ptr<int>()), (float)count, f32_opt(gamma), f32_opt(beta),
                     f32_opt_mut(rmean), f32_opt_mut(rvar), (float)momentum, (float)eps, st, st + Cp, st + 2 * Cp,
                     st + 3 * Cp, cur_stream());
}

void bn_reduce_bwd_finalize_t(const at::Tensor& part, int64_t nblk, int64_t C, int64_t Cp, const at::Tensor& tmp,
                              const at::Tensor& cnt, double count, const at::Tensor& stats,
                              const c10::optional<at::Tensor>& dgamma, const c10::optional<at::Tensor>& dbeta,
                              const at::Tensor& coef, double pscale) {
  CHECK_F32(part); CHECK_F64(tmp); CHECK_F32(stats); CHECK_F32(coef); CHECK_DEV(cnt);
  TORCH_CHECK(cnt.scalar_type() == at::kInt && cnt.numel() >= bn_rf_chunks(Cp), "cnt: int32 >= Cp/32 counters");
  TORCH_CHECK(part.numel() >= nblk * 2 * Cp, "partials too small");
  TORCH_CHECK(tmp.numel() >= (int64_t)bn_reduce_splits(nblk) * 2 * Cp, "tmp too small");
  TORCH_CHECK(coef.numel() == 3 * Cp && stats.numel() == 4 * Cp);
  const float* st = f32(stats);
  bn_reduce_bwd_finalize(f32(part), nblk, C, Cp, tmp.data_ptr<double>(), reinterpret_cast<unsigned*>(cnt.data_ptr<int>()),
                         (float)count, st, st + 3 * Cp, st + 2 * Cp, f32_opt_mut(dgamma), f32_opt_mut(dbeta), f32(coef),
                         (float)pscale, cur_stream());
}

void bn_act_apply_t(const at::Tensor& y, const at::Tensor& stats, const at::Tensor& z, int64_t P, int64_t Cp, bool relu) {
  CHECK_BF16(y); CHECK_BF16(z); CHECK_F32(stats);
  TORCH_CHECK(y.numel() == P * Cp && z.numel() == P * Cp && stats.numel() == 4 * Cp);
  const float* st = f32(stats);
  bn_act_apply(bf(y), st, st + Cp, bf(z), P, Cp, relu ? 1 : 0, cur_stream());
}

// the same pass with ReLU6 (MobileNetV2's BN -> ReLU6 in one pass)
void bn_act_apply_relu6_t(const at::Tensor& y, const at::Tensor& stats, const at::Tensor& z, int64_t P, int64_t Cp) {
  CHECK_BF16(y); CHECK_BF16(z); CHECK_F32(stats);
  TORCH_CHECK(y.numel() == P * Cp && z.numel() == P * Cp && stats.numel() == 4 * Cp);
  const float* st = f32(stats);
  bn_act_apply(bf(y), st, st + Cp, bf(z), P, Cp, 2, cur_stream());
}

void bn_add_act_t(const at::Tensor& y, const at::Tensor& sa, bool relu_a, const at::Tensor& x,
                  const c10::optional<at::Tensor>& sb, bool relu_b, const at::Tensor& z, bool relu) {
  CHECK_BF16(y); CHECK_BF16(x); CHECK_BF16(z); CHECK_F32(sa);
  const int64_t Cp = y.size(-1), P = y.numel() / Cp;
  TORCH_CHECK(Cp % 8 == 0 && x.numel() == P * Cp && z.numel() == P * Cp && sa.numel() == 4 * Cp, "bn_add_act shapes");
  const float* a = f32(sa);
  const float* b = nullptr;
  if (sb.has_value() && sb->defined()) {
    CHECK_F32(*sb);
    TORCH_CHECK(sb->numel() == 4 * Cp, "bn_add_act: identity BN stats");
    b = sb->data_ptr<float>();
  }
  bn_add_act(bf(y), a, a + Cp, relu_a ? 1 : 0, bf(x), b, b ? b + Cp : nullptr, relu_b ? 1 : 0, bf(z), P, (int)Cp,
             relu ? 1 : 0, cur_stream());
}

void bn_act_bwd_partial_t(const at::Tensor& dz, const at::Tensor& y, const at::Tensor& stats, const at::Tensor& part,
                          int64_t P, int64_t Cp, bool relu) {
  CHECK_BF16(dz); CHECK_BF16(y); CHECK_F32(stats); CHECK_F32(part);
  TORCH_CHECK(dz.numel() == P * Cp && y.numel() == P * Cp && stats.numel() == 4 * Cp);
  TORCH_CHECK(part.numel() == bn_partial_blocks(P, Cp) * 2 * Cp, "part numel mismatch");
  const float* st = f32(stats);
  bn_act_bwd_partial(bf(dz), bf(y), st, st + Cp, st + 2 * Cp, f32(part), P, Cp, relu ? 1 : 0, cur_stream());
}

void bn_bwd_finalize_t(const at::Tensor& tmp, int64_t C, int64_t Cp, double count, const at::Tensor& stats,
                       const c10::optional<at::Tensor>& dgamma, const c10::optional<at::Tensor>& dbeta,
                       const at::Tensor& coef, double pscale) {
  CHECK_F64(tmp); CHECK_F32(stats); CHECK_F32(coef);
  TORCH_CHECK(coef.numel() == 3 * Cp && stats.numel() == 4 * Cp && tmp.numel() % (2 * Cp) == 0);
  const float* st = f32(stats);
  bn_bwd_finalize(tmp.data_ptr<double>(), (int)(tmp.numel() / (2 * Cp)), C, Cp, (float)count, st, st + 3 * Cp,
                  st + 2 * Cp, f32_opt_mut(dgamma), f32_opt_mut(dbeta), f32(coef), (float)pscale, cur_stream());
}

void bn_act_bwd_apply_part_t(const at::Tensor& dz, const at::Tensor& y, const at::Tensor& stats, const at::Tensor& coef,
                             const at::Tensor& dy, const at::Tensor& y2, const at::Tensor& stats2, bool relu2,
                             const at::Tensor& part, int64_t P, int64_t Cp, bool relu) {
  CHECK_BF16(dz); CHECK_BF16(y); CHECK_BF16(dy); CHECK_BF16(y2); CHECK_F32(stats); CHECK_F32(coef);
  CHECK_F32(stats2); CHECK_F32(part);
  TORCH_CHECK(dz.numel() == P * Cp && y.numel() == P * Cp && dy.numel() == P * Cp && y2.numel() == P * Cp);
  TORCH_CHECK(stats.numel() == 4 * Cp && stats2.numel() == 4 * Cp && coef.numel() == 3 * Cp, "stats / coef rows");
  TORCH_CHECK(part.numel() == bn_partial_blocks(P, Cp) * 2 * Cp, "part numel mismatch");
  const float* st = f32(stats);
  const float* st2 = f32(stats2);
  bn_act_bwd_apply_part(bf(dz), bf(y), st, st + Cp, f32(coef), bf(dy), bf(y2), st2, st2 + Cp, st2 + 2 * Cp,
                        relu2 ? 1 : 0, f32(part), P, Cp, relu ? 1 : 0, cur_stream());
}

void bn_act_bwd_apply_t(const at::Tensor& dz, const at::Tensor& y, const at::Tensor& stats, const at::Tensor& coef,
                        const at::Tensor& dy, int64_t P, int64_t Cp, bool relu) {
  CHECK_BF16(dz); CHECK_BF16(y); CHECK_BF16(dy); CHECK_F32(stats); CHECK_F32(coef);
  TORCH_CHECK(dz.numel() == P * Cp && y.numel() == P * Cp && dy.numel() == P * Cp);
  const float* st = f32(stats);
  bn_act_bwd_apply(bf(dz), bf(y), st, st + Cp, f32(coef), bf(dy), P, Cp, relu ? 1 : 0, cur_stream());
}

// DUCK tail backward passes (bn.hip): out_bn (dz, ys, stats, coef) + k branch-last BNs (y_i, stats_i
// [, coef_i, dy_i]); part = fp32 [k, bn_tail_blocks(P, Cp), 2, Cp]
static void tail_check(const at::Tensor& dz, const at::Tensor& ys, const at::Tensor& ostats, const at::Tensor& ocoef,
                       const std::vector<at::Tensor>& y, const std::vector<at::Tensor>& st, int64_t P, int64_t Cp) {
  CHECK_BF16(dz); CHECK_BF16(ys); CHECK_F32(ostats); CHECK_F32(ocoef);
  TORCH_CHECK(Cp % 8 == 0 && Cp <= kTailMaxCp, "tail passes: Cp a multiple of 8, <= ", kTailMaxCp);
  TORCH_CHECK(!y.empty() && (int)y.size() <= kTailMax && st.size() == y.size(), "1..6 branches");
  TORCH_CHECK(dz.numel() == P * Cp && ys.numel() == P * Cp && ostats.numel() == 4 * Cp && ocoef.numel() == 3 * Cp);
  for (size_t i = 0; i < y.size(); ++i) {
    CHECK_BF16(y[i]); CHECK_F32(st[i]);
    TORCH_CHECK(y[i].numel() == P * Cp && st[i].numel() == 4 * Cp, "branch tensor / stats size mismatch");
  }
}

void bn_tail_partial_t(const at::Tensor& dz, const at::Tensor& ys, const at::Tensor& ostats, const at::Tensor& ocoef,
                       bool orelu, std::vector<at::Tensor> y, std::vector<at::Tensor> st, int64_t relu_mask,
                       const at::Tensor& part, int64_t P, int64_t Cp) {
  tail_check(dz, ys, ostats, ocoef, y, st, P, Cp);
  CHECK_F32(part);
  TORCH_CHECK(part.numel() == (int64_t)y.size() * bn_tail_blocks(P, Cp) * 2 * Cp, "part: [k, bn_tail_blocks, 2, Cp]");
  std::vector<const uint16_t*> yp;
  std::vector<const float*> sp;
  for (size_t i = 0; i < y.size(); ++i) { yp.push_back(bf(y[i])); sp.push_back(f32(st[i])); }
  bn_tail_partial(bf(dz), bf(ys), f32(ostats), f32(ocoef), orelu ? 1 : 0, (int)y.size(), yp.data(), sp.data(),
                  (unsigned)relu_mask, f32(part), P, Cp, cur_stream());
}

void bn_tail_apply_t(const at::Tensor& dz, const at::Tensor& ys, const at::Tensor& ostats, const at::Tensor& ocoef,
                     bool orelu, std::vector<at::Tensor> y, std::vector<at::Tensor> st, std::vector<at::Tensor> coef,
                     int64_t relu_mask, std::vector<at::Tensor> dy, int64_t P, int64_t Cp,
                     const c10::optional<at::Tensor>& g) {
  tail_check(dz, ys, ostats, ocoef, y, st, P, Cp);
  TORCH_CHECK(coef.size() == y.size() && dy.size() == y.size(), "coef / dy per branch");
  std::vector<const uint16_t*> yp;
  std::vector<const float*> sp, cp;
  std::vector<uint16_t*> dp;
  bool deferred = false;
  for (size_t i = 0; i < y.size(); ++i) {
    CHECK_F32(coef[i]); CHECK_BF16(dy[i]);
    // an empty dy: the branch's data-gradient is deferred (rebuilt from g by its producer)
    TORCH_CHECK(coef[i].numel() == 3 * Cp && (dy[i].numel() == P * Cp || dy[i].numel() == 0), "coef / dy size mismatch");
    deferred |= dy[i].numel() == 0;
    yp.push_back(bf(y[i])); sp.push_back(f32(st[i])); cp.push_back(f32(coef[i]));
    dp.push_back(dy[i].numel() == 0 ? nullptr : bf(dy[i]));
  }
  uint16_t* gp = nullptr;
  if (g.has_value() && g->defined()) {
    CHECK_BF16(*g); TORCH_CHECK(g->numel() == P * Cp, "g numel");
    gp = bf(*g);
  }
  TORCH_CHECK(!deferred || gp != nullptr, "deferred branches need g");
  bn_tail_apply(bf(dz), bf(ys), f32(ostats), f32(ocoef), orelu ? 1 : 0, (int)y.size(), yp.data(), sp.data(), cp.data(),
                (unsigned)relu_mask, dp.data(), P, Cp, cur_stream(), gp);
}

void nchw_to_nhwc_t(const at::Tensor& x, const at::Tensor& y, int64_t Cp) {
  CHECK_F32(x); CHECK_BF16(y);
  TORCH_CHECK(x.dim() == 4, "x must be NCHW");
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(y.numel() == (int64_t)N * H * W * Cp && C <= Cp);
  nchw_to_nhwc(f32(x), bf(y), N, C, H, W, Cp, cur_stream());
}

void nhwc_to_nchw_t(const at::Tensor& x, const at::Tensor& y, int64_t Cp) {
  CHECK_BF16(x); CHECK_F32(y);
  TORCH_CHECK(y.dim() == 4, "y must be NCHW");
  const int N = y.size(0), C = y.size(1), H = y.size(2), W = y.size(3);
  TORCH_CHECK(x.numel() == (int64_t)N * H * W * Cp && C <= Cp);
  nhwc_to_nchw(bf(x), f32(y), N, C, H, W, Cp, cur_stream());
}

void up2_add_t(const at::Tensor& low, const at::Tensor& skip, const at::Tensor& out, int64_t N, int64_t h, int64_t w,
               int64_t Cp, OptTensors coefs, int64_t relu_mask) {
  CHECK_BF16(low); CHECK_BF16(skip); CHECK_BF16(out);
  TORCH_CHECK(low.numel() == N * h * w * Cp && skip.numel() == 4 * N * h * w * Cp && out.numel() == skip.numel());
  const float* cf[2];
  fill_coefs(coefs, 2, {Cp, Cp}, cf);   // [low, skip]
  up2_add(bf(low), bf(skip), bf(out), N, h, w, Cp, cf[0], (int)(relu_mask & 1), cf[1], (int)((relu_mask >> 1) & 1),
          cur_stream());
}

void pool2_sum_t(const at::Tensor& g, const at::Tensor& out, int64_t N, int64_t h, int64_t w, int64_t Cp) {
  CHECK_BF16(g); CHECK_BF16(out);
  TORCH_CHECK(out.numel() == N * h * w * Cp && g.numel() == 4 * out.numel());
  pool2_sum(bf(g), bf(out), N, h, w, Cp, cur_stream());
}

void add_n_t(std::vector<at::Tensor> inputs, const at::Tensor& out, OptTensors coefs, int64_t relu_mask) {
  TORCH_CHECK(!inputs.empty() && (int)inputs.size() <= kMaxSumInputs);
  CHECK_BF16(out);
  TORCH_CHECK(out.numel() % 8 == 0 && out.dim() >= 1);
  const int64_t Cp = out.size(-1);
  TORCH_CHECK(Cp % 8 == 0, "channel dim must be a multiple of 8");
  std::vector<const uint16_t*> ptrs;
  for (auto& t : inputs) { CHECK_BF16(t); TORCH_CHECK(t.numel() == out.numel()); ptrs.push_back(bf(t)); }
  const float* cf[kMaxSumInputs];
  fill_coefs(coefs, (int)ptrs.size(), std::vector<int64_t>(ptrs.size(), Cp), cf);
  add_n(ptrs.data(), cf, (unsigned)relu_mask, (int)ptrs.size(), bf(out), out.numel(), (int)Cp, cur_stream());
}

inline uint8_t* u8(const at::Tensor& t) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == at::kByte, "idx must be a contiguous uint8 GPU tensor");
  return t.data_ptr<uint8_t>();
}

void maxpool_fwd_t(const at::Tensor& x, const at::Tensor& y, const at::Tensor& idx, int64_t k, int64_t s, int64_t p) {
  CHECK_BF16(x); CHECK_BF16(y);
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4 && x.size(0) == y.size(0) && x.size(3) == y.size(3) && x.size(3) % 8 == 0);
  TORCH_CHECK(idx.numel() == y.numel() && k >= 1 && k * k <= 255 && s >= 1 && 2 * p <= k);
  TORCH_CHECK(y.size(1) == (x.size(1) + 2 * p - k) / s + 1 && y.size(2) == (x.size(2) + 2 * p - k) / s + 1, "maxpool out shape");
  maxpool_fwd(bf(x), bf(y), u8(idx), x.size(0), x.size(1), x.size(2), y.size(1), y.size(2), x.size(3), k, s, p, cur_stream());
}

void maxpool_bwd_t(const at::Tensor& dy, const at::Tensor& idx, const at::Tensor& dx, int64_t k, int64_t s, int64_t p) {
  CHECK_BF16(dy); CHECK_BF16(dx);
  TORCH_CHECK(dy.dim() == 4 && dx.dim() == 4 && dy.size(3) == dx.size(3) && idx.numel() == dy.numel());
  TORCH_CHECK(dy.size(1) == (dx.size(1) + 2 * p - k) / s + 1 && dy.size(2) == (dx.size(2) + 2 * p - k) / s + 1, "maxpool shape");
  maxpool_bwd(bf(dy), u8(idx), bf(dx), dx.size(0), dx.size(1), dx.size(2), dy.size(1), dy.size(2), dx.size(3), k, s, p,
              cur_stream());
}

void up2_cat_t(const at::Tensor& low, const c10::optional<at::Tensor>& skip, const at::Tensor& out, int64_t Cl,
               int64_t Cs) {
  CHECK_BF16(low); CHECK_BF16(out);
  const int64_t N = low.size(0), h = low.size(1), w = low.size(2), Cpl = low.size(3), Cpo = out.size(3);
  TORCH_CHECK(out.size(0) == N && out.size(1) == 2 * h && out.size(2) == 2 * w && Cpo % 8 == 0 && Cpl % 8 == 0);
  TORCH_CHECK(Cl <= Cpl && Cl + Cs <= Cpo, "channel ranges");
  const uint16_t* sp = nullptr;
  int64_t Cps = 8;
  if (Cs > 0) {
    TORCH_CHECK(skip.has_value() && skip->defined(), "skip required when Cs > 0");
    CHECK_BF16(*skip);
    TORCH_CHECK(skip->size(0) == N && skip->size(1) == 2 * h && skip->size(2) == 2 * w && skip->size(3) >= Cs);
    Cps = skip->size(3);
    sp = bf(*skip);
  }
  up2_cat(bf(low), sp, bf(out), N, h, w, Cl, Cpl, Cs, Cps, Cpo, cur_stream());
}

void up2_cat_bwd_t(const at::Tensor& g, const at::Tensor& dlow, const c10::optional<at::Tensor>& dskip, int64_t Cl,
                   int64_t Cs) {
  CHECK_BF16(g); CHECK_BF16(dlow);
  const int64_t N = dlow.size(0), h = dlow.size(1), w = dlow.size(2), Cpl = dlow.size(3), Cpo = g.size(3);
  TORCH_CHECK(g.size(0) == N && g.size(1) == 2 * h && g.size(2) == 2 * w && Cl <= Cpl && Cl + Cs <= Cpo);
  uint16_t* dp = nullptr;
  int64_t Cps = 8;
  if (Cs > 0) {
    TORCH_CHECK(dskip.has_value() && dskip->defined());
    CHECK_BF16(*dskip);
    TORCH_CHECK(dskip->size(0) == N && dskip->size(1) == 2 * h && dskip->size(2) == 2 * w && dskip->size(3) >= Cs);
    Cps = dskip->size(3);
    dp = bf(*dskip);
  }
  up2_cat_bwd(bf(g), bf(dlow), dp, N, h, w, Cl, Cpl, Cs, Cps, Cpo, cur_stream());
}

void add_act_t(const at::Tensor& a, const at::Tensor& b, const at::Tensor& z, bool relu) {
  CHECK_BF16(a); CHECK_BF16(b); CHECK_BF16(z);
  TORCH_CHECK(a.numel() == b.numel() && a.numel() == z.numel() && a.numel() % 8 == 0);
  add_act(bf(a), bf(b), bf(z), a.numel(), relu ? 1 : 0, cur_stream());
}

void relu_bwd_t(const at::Tensor& dz, const at::Tensor& z, const at::Tensor& g) {
  CHECK_BF16(dz); CHECK_BF16(z); CHECK_BF16(g);
  TORCH_CHECK(dz.numel() == z.numel() && z.numel() == g.numel() && z.numel() % 8 == 0);
  relu_bwd(bf(dz), bf(z), bf(g), z.numel(), cur_stream());
}

// ---- inference glue (metrics.hip)
void bilinear_resize_t(const at::Tensor& x, const at::Tensor& y, bool align_corners) {
  CHECK_F32(x); CHECK_F32(y);
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4 && x.size(0) == y.size(0) && x.size(1) == y.size(1));
  bilinear_resize(f32(x), f32(y), x.size(0) * x.size(1), x.size(2), x.size(3), y.size(2), y.size(3),
                  align_corners ? 1 : 0, cur_stream());
}

void colorize_t(const at::Tensor& logits, const at::Tensor& lut, const at::Tensor& rgb) {
  CHECK_F32(logits);
  TORCH_CHECK(lut.is_cuda() && lut.scalar_type() == at::kByte && lut.is_contiguous() && lut.size(1) == 3);
  TORCH_CHECK(rgb.is_cuda() && rgb.scalar_type() == at::kByte && rgb.is_contiguous());
  const int64_t N = logits.size(0), C = logits.size(1), HW = logits.size(2) * logits.size(3);
  TORCH_CHECK(lut.size(0) >= (C == 1 ? 2 : C) && rgb.numel() == N * HW * 3);
  colorize(f32(logits), lut.data_ptr<uint8_t>(), rgb.data_ptr<uint8_t>(), N, C, HW, cur_stream());
}

// ---- GPU augmentation (augment.hip)
void aug_batch_t(const at::Tensor& images, const at::Tensor& masks, const at::Tensor& meta, const at::Tensor& ip,
                 const at::Tensor& fp, const at::Tensor& work, const at::Tensor& mean, const at::Tensor& out,
                 const at::Tensor& mask_out, std::vector<int64_t> stages, std::vector<int64_t> contrast_stages,
                 std::vector<double> norm_mean, std::vector<double> norm_std) {
  TORCH_CHECK(images.is_cuda() && images.scalar_type() == at::kByte && images.is_contiguous());
  TORCH_CHECK(masks.is_cuda() && masks.scalar_type() == at::kByte && masks.is_contiguous());
  CHECK_I64(meta); CHECK_I64(mask_out); CHECK_F32(fp); CHECK_F32(work); CHECK_F32(mean); CHECK_F32(out);
  TORCH_CHECK(ip.is_cuda() && ip.scalar_type() == at::kInt && ip.is_contiguous());
  TORCH_CHECK(out.dim() == 4 && out.size(1) == 3, "out must be [B, 3, H, W]");
  const int B = out.size(0), H = out.size(2), W = out.size(3);
  // mean: [B] floats, then (8-B aligned) the fp64 slice partials of the gray mean
  const int64_t poff = ((int64_t)B + 1) / 2 * 2;
  TORCH_CHECK(ip.numel() == (int64_t)B * kAugIParams && fp.numel() == (int64_t)B * 4 &&
              mean.numel() >= poff + 2 * (int64_t)aug_gray_scratch_doubles(B), "aug: mean [B + gray partials]");
  TORCH_CHECK(work.numel() == (int64_t)B * H * W * 3 && mask_out.numel() == (int64_t)B * H * W);
  TORCH_CHECK(meta.dim() == 2 && meta.size(1) == 4 && norm_mean.size() == 3 && norm_std.size() == 3);
  auto s = cur_stream();
  aug_geometry(images.data_ptr<uint8_t>(), masks.data_ptr<uint8_t>(), meta.data_ptr<int64_t>(), ip.data_ptr<int>(),
               f32(work), mask_out.data_ptr<int64_t>(), B, H, W, s);
  for (size_t k = 0; k < stages.size(); ++k) {
    const int st = (int)stages[k];
    TORCH_CHECK(st >= 0 && st < 4);
    if (std::find(contrast_stages.begin(), contrast_stages.end(), stages[k]) != contrast_stages.end())
      aug_gray_mean(f32(work), f32(mean), reinterpret_cast<double*>(f32(mean) + poff), B, H * W, s);
    aug_color(f32(work), ip.data_ptr<int>(), f32(fp), f32(mean), B, H * W, st, s);
  }
  const float m3[3] = {(float)norm_mean[0], (float)norm_mean[1], (float)norm_mean[2]};
  const float s3[3] = {(float)norm_std[0], (float)norm_std[1], (float)norm_std[2]};
  aug_finalize(f32(work), ip.data_ptr<int>(), f32(out), B, H * W, m3, s3, s);
}

void scale_f32_t(const at::Tensor& x, const c10::optional<at::Tensor>& scalar, double mult) {
  CHECK_F32(x);
  scale_f32(f32(x), f32_opt(scalar), (float)mult, x.numel(), cur_stream());
}

int64_t ce_blocks_t(int64_t P) { return ce_blocks(P); }

void ce_fwd_bwd_t(const at::Tensor& logits, const at::Tensor& target, const c10::optional<at::Tensor>& weight,
                  const at::Tensor& grad, const c10::optional<at::Tensor>& pix_loss, const at::Tensor& part,
                  int64_t ignore_index) {
  CHECK_F32(logits); CHECK_I64(target); CHECK_F32(grad); CHECK_F32(part);
  TORCH_CHECK(logits.dim() == 4, "logits must be NCHW");
  const int N = logits.size(0), C = logits.size(1);
  const long HW = logits.size(2) * logits.size(3);
  TORCH_CHECK(target.numel() == (int64_t)N * HW && grad.numel() == logits.numel());
  TORCH_CHECK(part.numel() == 2 * ce_blocks((long)N * HW));
  float* pl = f32_opt_mut(pix_loss);
  if (pl) TORCH_CHECK(pix_loss->numel() == (int64_t)N * HW);
  ce_fwd_bwd(f32(logits), target.data_ptr<int64_t>(), f32_opt(weight), f32(grad), pl, f32(part), N, C, HW,
             (int)ignore_index, cur_stream());
}

void ohem_select_t(const at::Tensor& pix, const at::Tensor& target, double thr, int64_t ignore_index,
                   const at::Tensor& bpart, const at::Tensor& state, const at::Tensor& hist, const at::Tensor& loss) {
  CHECK_F32(pix); CHECK_I64(target); CHECK_F32(bpart); CHECK_F32(loss); CHECK_DEV(state); CHECK_DEV(hist);
  const long P = pix.numel();
  TORCH_CHECK(target.numel() == P && bpart.numel() == 3 * ce_blocks(P) && loss.numel() == 1);
  TORCH_CHECK(state.scalar_type() == at::kInt && state.numel() == ohem_state_words(), "state: int32 [ohem_state_words]");
  TORCH_CHECK(hist.scalar_type() == at::kInt && hist.numel() == 256, "hist: int32 [256]");
  ohem_select(f32(pix), target.data_ptr<int64_t>(), P, (float)thr, (int)ignore_index, f32(bpart),
              reinterpret_cast<unsigned*>(state.data_ptr<int>()), reinterpret_cast<unsigned*>(hist.data_ptr<int>()),
              f32(loss), cur_stream());
}

void ohem_backward_t(const at::Tensor& grad, const at::Tensor& pix, const at::Tensor& state, const at::Tensor& gup) {
  CHECK_F32(grad); CHECK_F32(pix); CHECK_F32(gup); CHECK_DEV(state);
  TORCH_CHECK(grad.dim() == 4 && pix.numel() == grad.size(0) * grad.size(2) * grad.size(3) && gup.numel() == 1);
  ohem_backward(f32(grad), f32(pix), reinterpret_cast<const unsigned*>(state.data_ptr<int>()), f32(gup), grad.size(0),
                grad.size(1), grad.size(2) * grad.size(3), cur_stream());
}

void kd_kl_fwd_bwd_t(const at::Tensor& s, const at::Tensor& t, const at::Tensor& grad, const at::Tensor& part,
                     double T) {
  CHECK_F32(s); CHECK_F32(t); CHECK_F32(grad); CHECK_F32(part);
  TORCH_CHECK(s.dim() == 4 && s.sizes() == t.sizes() && grad.numel() == s.numel());
  const int N = s.size(0), C = s.size(1);
  const long HW = s.size(2) * s.size(3);
  TORCH_CHECK(part.numel() == ce_blocks((long)N * HW));
  kd_kl_fwd_bwd(f32(s), f32(t), f32(grad), f32(part), N, C, HW, (float)T, cur_stream());
}

void mse_fwd_bwd_t(const at::Tensor& s, const at::Tensor& t, const at::Tensor& grad, const at::Tensor& part) {
  CHECK_F32(s); CHECK_F32(t); CHECK_F32(grad); CHECK_F32(part);
  TORCH_CHECK(s.sizes() == t.sizes() && grad.numel() == s.numel() && part.numel() == ce_blocks(s.numel()));
  mse_fwd_bwd(f32(s), f32(t), f32(grad), f32(part), s.numel(), cur_stream());
}

void bce_dice_stats_t(const at::Tensor& x, const at::Tensor& t, const at::Tensor& part) {
  CHECK_F32(x); CHECK_F32(t); CHECK_F32(part);
  TORCH_CHECK(x.dim() >= 2 && x.numel() == t.numel(), "logits [N, ...] and targets of the same numel");
  const int N = x.size(0);
  const long HW = x.numel() / N;
  TORCH_CHECK(part.numel() == (int64_t)N * bce_dice_splits(HW) * 4, "part must be [N, splits, 4]");
  bce_dice_stats(f32(x), f32(t), f32(part), N, HW, cur_stream());
}

void bce_dice_grad_t(const at::Tensor& x, const at::Tensor& t, const at::Tensor& coef, const at::Tensor& gup,
                     const at::Tensor& grad, double bw, double dw) {
  CHECK_F32(x); CHECK_F32(t); CHECK_F32(coef); CHECK_F32(gup); CHECK_F32(grad);
  const int N = x.size(0);
  const long HW = x.numel() / N;
  TORCH_CHECK(t.numel() == x.numel() && grad.numel() == x.numel() && coef.numel() == 2 * N && gup.numel() == 1);
  bce_dice_grad(f32(x), f32(t), f32(coef), f32(gup), f32(grad), N, HW, (float)bw, (float)dw, cur_stream());
}

int64_t bce_dice_splits_t(int64_t HW) { return bce_dice_splits(HW); }

static const float* amp_ptr(const c10::optional<at::Tensor>& amp) {
  if (amp.has_value()) { CHECK_F32(*amp); TORCH_CHECK(amp->numel() >= 4); }
  return f32_opt(amp);
}

void adam_step_t(const at::Tensor& p, const at::Tensor& g, const at::Tensor& m, const at::Tensor& v,
                 const at::Tensor& hyper, bool adamw, const c10::optional<at::Tensor>& amp) {
  CHECK_F32(p); CHECK_F32(g); CHECK_F32(m); CHECK_F32(v); CHECK_F32(hyper);
  TORCH_CHECK(g.numel() == p.numel() && m.numel() == p.numel() && v.numel() == p.numel() && hyper.numel() >= 8);
  adam_step(f32(p), f32(g), f32(m), f32(v), f32(hyper), p.numel(), adamw ? 1 : 0, amp_ptr(amp), cur_stream());
}

void sgd_step_t(const at::Tensor& p, const at::Tensor& g, const at::Tensor& buf, const at::Tensor& hyper,
                const c10::optional<at::Tensor>& amp) {
  CHECK_F32(p); CHECK_F32(g); CHECK_F32(buf); CHECK_F32(hyper);
  TORCH_CHECK(g.numel() == p.numel() && buf.numel() == p.numel() && hyper.numel() >= 4);
  sgd_step(f32(p), f32(g), f32(buf), f32(hyper), p.numel(), amp_ptr(amp), cur_stream());
}

void amp_check_t(const at::Tensor& g, const at::Tensor& amp) {
  CHECK_F32(g); CHECK_F32(amp);
  TORCH_CHECK(amp.numel() >= 4);
  amp_check(f32(g), g.numel(), f32(amp), cur_stream());
}

void amp_update_t(const at::Tensor& amp, double growth, double backoff, int64_t interval) {
  CHECK_F32(amp);
  TORCH_CHECK(amp.numel() >= 4 && interval >= 1);
  amp_update(f32(amp), (float)growth, (float)backoff, (int)interval, cur_stream());
}

void ema_update_t(const at::Tensor& ema, const at::Tensor& model, const at::Tensor& hyper) {
  CHECK_F32(ema); CHECK_F32(model); CHECK_F32(hyper);
  TORCH_CHECK(ema.numel() == model.numel());
  ema_update(f32(ema), f32(model), f32(hyper), ema.numel(), cur_stream());
}

void confmat_update_t(const at::Tensor& logits, const at::Tensor& target, const at::Tensor& confmat,
                      int64_t ignore_index) {
  CHECK_F32(logits); CHECK_I64(target); CHECK_I64(confmat);
  TORCH_CHECK(logits.dim() == 4);
  const int N = logits.size(0), C = logits.size(1);
  const long HW = logits.size(2) * logits.size(3);
  TORCH_CHECK(C * C <= 1024 && confmat.numel() == (int64_t)C * C && target.numel() == (int64_t)N * HW);
  confmat_update(f32(logits), target.data_ptr<int64_t>(), confmat.data_ptr<int64_t>(), N, C, HW, (int)ignore_index,
                 cur_stream());
}


// ---- decoder-hub ops (decoder.hip)
void resize_bilinear_t(const at::Tensor& x, const at::Tensor& y, double sh, double sw, bool align, bool accum,
                       bool backward) {
  CHECK_BF16(x); CHECK_BF16(y);
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4 && x.size(0) == y.size(0) && x.size(3) == y.size(3) && x.size(3) % 8 == 0,
              "resize: NHWC bf16 maps with equal N and padded C");
  // forward: x [N,IH,IW,C] -> y [N,OH,OW,C]; backward: x = dY [N,OH,OW,C] -> y = dX [N,IH,IW,C]
  if (!backward)
    resize_bilinear_fwd(bf(x), bf(y), x.size(0), x.size(1), x.size(2), y.size(1), y.size(2), x.size(3), (float)sh,
                        (float)sw, align ? 1 : 0, accum ? 1 : 0, cur_stream());
  else
    resize_bilinear_bwd(bf(x), bf(y), y.size(0), y.size(1), y.size(2), x.size(1), x.size(2), x.size(3), (float)sh,
                        (float)sw, align ? 1 : 0, cur_stream());
}

int64_t nc_sums_blocks_t(int64_t HW, int64_t Cp) { return nc_sums_blocks(HW, (int)Cp); }

void nc_sums_t(const at::Tensor& x, const c10::optional<at::Tensor>& dz, const c10::optional<at::Tensor>& tab,
               bool relu, const at::Tensor& part) {
  CHECK_BF16(x); CHECK_F32(part);
  TORCH_CHECK(x.dim() == 4 && x.size(3) % 8 == 0 && x.size(3) <= 2048, "nc_sums: NHWC bf16, C <= 2048");
  const int N = x.size(0), Cp = x.size(3);
  const long HW = x.size(1) * x.size(2);
  TORCH_CHECK(part.dim() == 4 && part.size(0) == N && part.size(2) == 2 && part.size(3) == Cp, "part [N][nblk][2][Cp]");
  const uint16_t* g = nullptr;
  if (dz.has_value() && dz->defined()) {
    CHECK_BF16(*dz);
    TORCH_CHECK(dz->sizes() == x.sizes(), "dz shape");
    g = bf(*dz);
    TORCH_CHECK(tab.has_value() && tab->numel() >= (int64_t)N * 4 * Cp, "nc_sums backward needs the [N][4][Cp] table");
  }
  nc_sums(bf(x), g, f32_opt(tab), relu ? 1 : 0, N, HW, Cp, f32(part), part.size(1), cur_stream());
}

void gn_finalize_t(const at::Tensor& part, int64_t C, int64_t G, double eps, const c10::optional<at::Tensor>& gamma,
                   const c10::optional<at::Tensor>& beta, int64_t HW, const at::Tensor& tab) {
  CHECK_F32(part); CHECK_F32(tab);
  const int N = part.size(0), nblk = part.size(1), Cp = part.size(3);
  TORCH_CHECK(C % G == 0 && C <= Cp && tab.numel() == (int64_t)N * 4 * Cp, "gn_finalize shapes");
  gn_finalize(f32(part), nblk, N, C, Cp, G, (float)eps, f32_opt(gamma), f32_opt(beta), HW, f32(tab), cur_stream());
}

void gn_bwd_finalize_t(const at::Tensor& part, int64_t C, int64_t G, const c10::optional<at::Tensor>& gamma,
                       const at::Tensor& tab, int64_t HW, const c10::optional<at::Tensor>& dgamma,
                       const c10::optional<at::Tensor>& dbeta, const at::Tensor& coef) {
  CHECK_F32(part); CHECK_F32(tab); CHECK_F32(coef);
  const int N = part.size(0), nblk = part.size(1), Cp = part.size(3);
  TORCH_CHECK(C % G == 0 && coef.numel() == (int64_t)N * 3 * Cp, "gn_bwd_finalize shapes");
  gn_bwd_finalize(f32(part), nblk, N, C, Cp, G, f32_opt(gamma), f32(tab), HW, f32_opt_mut(dgamma), f32_opt_mut(dbeta),
                  f32(coef), cur_stream());
}

void affine_nc_t(const at::Tensor& x, const at::Tensor& tab, int64_t rows, const at::Tensor& z, bool relu) {
  CHECK_BF16(x); CHECK_F32(tab); CHECK_BF16(z);
  TORCH_CHECK(x.dim() == 4 && z.sizes() == x.sizes() && tab.numel() >= x.size(0) * rows * x.size(3), "affine_nc shapes");
  affine_nc(bf(x), f32(tab), rows, bf(z), x.size(0), x.size(1) * x.size(2), x.size(3), relu ? 1 : 0, cur_stream());
}

void affine_nc_bwd_t(const at::Tensor& dz, const at::Tensor& x, const at::Tensor& tab, const at::Tensor& coef,
                     const at::Tensor& dx, bool relu) {
  CHECK_BF16(dz); CHECK_BF16(x); CHECK_F32(tab); CHECK_F32(coef); CHECK_BF16(dx);
  TORCH_CHECK(x.dim() == 4 && dz.sizes() == x.sizes() && dx.sizes() == x.sizes(), "affine_nc_bwd shapes");
  TORCH_CHECK(tab.numel() >= x.size(0) * 4 * x.size(3) && coef.numel() >= x.size(0) * 3 * x.size(3), "tables");
  affine_nc_bwd(bf(dz), bf(x), f32(tab), f32(coef), bf(dx), x.size(0), x.size(1) * x.size(2), x.size(3),
                relu ? 1 : 0, cur_stream());
}

void adaptive_avgpool_t(const at::Tensor& x, const at::Tensor& y, bool backward) {
  CHECK_BF16(x); CHECK_BF16(y);
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4 && x.size(0) == y.size(0) && x.size(3) == y.size(3) && x.size(3) % 8 == 0 &&
              x.size(3) <= 2048, "adaptive_avgpool: NHWC bf16, C <= 2048");
  if (!backward)   // x [N,H,W,C] -> y [N,OH,OW,C]
    adaptive_avgpool_fwd(bf(x), bf(y), x.size(0), x.size(1), x.size(2), y.size(1), y.size(2), x.size(3), cur_stream());
  else             // x = dY [N,OH,OW,C] -> y = dX [N,H,W,C]
    adaptive_avgpool_bwd(bf(x), bf(y), y.size(0), y.size(1), y.size(2), x.size(1), x.size(2), x.size(3), cur_stream());
}

void dwconv_fwd_t(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias, const at::Tensor& y,
                  std::vector<int64_t> dy, std::vector<int64_t> dx) {
  CHECK_BF16(x); CHECK_F32(w); CHECK_BF16(y);
  const int T = dy.size();
  TORCH_CHECK(T >= 1 && T <= kMaxTaps && (int)dx.size() == T, "dwconv taps");
  TORCH_CHECK(x.dim() == 4 && y.sizes() == x.sizes() && x.size(3) % 8 == 0 && w.numel() == (int64_t)T * x.size(3),
              "dwconv: stride-1 NHWC bf16, w [T][Cp]");
  int ty[kMaxTaps], tx[kMaxTaps];
  for (int t = 0; t < T; ++t) { ty[t] = dy[t]; tx[t] = dx[t]; }
  dwconv_fwd(bf(x), f32(w), f32_opt(bias), bf(y), x.size(0), x.size(1), x.size(2), x.size(3), T, ty, tx, cur_stream());
}

int64_t dwconv_wgrad_blocks_t(int64_t P, int64_t Cp) { return dwconv_wgrad_blocks(P, (int)Cp); }

void dwconv_wgrad_t(const at::Tensor& x, const at::Tensor& dyv, const at::Tensor& part, std::vector<int64_t> dy,
                    std::vector<int64_t> dx) {
  CHECK_BF16(x); CHECK_BF16(dyv); CHECK_F32(part);
  const int T = dy.size();
  TORCH_CHECK(T >= 1 && T <= 9 && (int)dx.size() == T, "dwconv_wgrad: up to 9 taps");
  TORCH_CHECK(dyv.sizes() == x.sizes() && part.dim() == 3 && part.size(1) == T + 1 && part.size(2) == x.size(3),
              "dwconv_wgrad: part [nblk][T+1][Cp]");
  int ty[kMaxTaps], tx[kMaxTaps];
  for (int t = 0; t < T; ++t) { ty[t] = dy[t]; tx[t] = dx[t]; }
  const int rc = dwconv_wgrad(bf(x), bf(dyv), f32(part), part.size(0), x.size(0), x.size(1), x.size(2), x.size(3), T,
                              ty, tx, cur_stream());
  TORCH_CHECK(rc == 0, "dwconv_wgrad: no instantiation");
}

void relu6_t(const at::Tensor& x, const at::Tensor& y) {
  CHECK_BF16(x); CHECK_BF16(y);
  TORCH_CHECK(x.numel() == y.numel() && x.numel() % 8 == 0, "relu6: same numel, multiple of 8");
  relu6(bf(x), bf(y), x.numel(), cur_stream());
}

void bn_aug_mask_t(const at::Tensor& x, const at::Tensor& stats, const at::Tensor& out, int64_t C) {
  CHECK_BF16(x); CHECK_BF16(out);
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous() && x.size(-1) == 8 && out.numel() == x.numel(),
              "bn_aug_mask: contiguous 8-channel pixels, out like x");
  TORCH_CHECK(C >= 1 && C <= 4, "bn_aug_mask: 1 <= C <= 4 (2C channels of 8)");
  TORCH_CHECK(stats.scalar_type() == at::kFloat && stats.is_contiguous() && stats.numel() >= 16 && stats.size(-1) == 8,
              "bn_aug_mask: stats fp32 [>=2][8]");
  bn_aug_mask(bf(x), f32(stats), bf(out), x.numel() / 8, (int)C, cur_stream());
}

void relu6_bwd_t(const at::Tensor& dy, const at::Tensor& y, const at::Tensor& dx) {
  CHECK_BF16(dy); CHECK_BF16(y); CHECK_BF16(dx);
  TORCH_CHECK(dy.numel() == y.numel() && dx.numel() == y.numel() && y.numel() % 8 == 0, "relu6_bwd: shapes");
  relu6_bwd(bf(dy), bf(y), bf(dx), y.numel(), cur_stream());
}

// ---- gconv.hip: grouped convolution (NHWC bf16, fp32 weights [T][C][CG]) -------------------------------
static void gconv_check(const at::Tensor& x, const at::Tensor& y, int64_t CG, const std::vector<int64_t>& dy,
                        const std::vector<int64_t>& dx) {
  CHECK_BF16(x); CHECK_BF16(y);
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4 && x.size(0) == y.size(0) && x.size(3) == y.size(3), "gconv: NHWC maps");
  TORCH_CHECK(x.size(3) % 8 == 0 && x.size(3) % CG == 0, "gconv: C % 8 == 0 and C % CG == 0");
  TORCH_CHECK(CG == 1 || CG == 2 || CG == 4 || CG == 8 || CG == 16 || CG == 32 || CG == 64, "gconv: CG");
  TORCH_CHECK(dy.size() == dx.size() && !dy.empty() && (int)dy.size() <= kMaxTaps, "gconv: taps");
}

void gconv_fwd_t(const at::Tensor& x, const at::Tensor& w, const at::Tensor& y, int64_t CG, int64_t stride,
                 std::vector<int64_t> dy, std::vector<int64_t> dx) {
  gconv_check(x, y, CG, dy, dx);
  CHECK_F32(w);
  const int C = x.size(3), T = dy.size();
  TORCH_CHECK(w.numel() == (int64_t)T * C * CG, "gconv: w [T][C][CG]");
  int ty[kMaxTaps], tx[kMaxTaps];
  for (int t = 0; t < T; ++t) { ty[t] = dy[t]; tx[t] = dx[t]; }
  const int rc = gconv_fwd(bf(x), f32(w), bf(y), x.size(0), x.size(1), x.size(2), y.size(1), y.size(2), C, CG, stride, T,
                           ty, tx, cur_stream());
  TORCH_CHECK(rc == 0, "gconv_fwd: no instantiation");
}

void gconv_dgrad_t(const at::Tensor& g, const at::Tensor& w, const at::Tensor& dxo, int64_t CG, int64_t stride,
                   std::vector<int64_t> dy, std::vector<int64_t> dx) {
  gconv_check(dxo, g, CG, dy, dx);
  CHECK_F32(w);
  const int C = dxo.size(3), T = dy.size();
  TORCH_CHECK(w.numel() == (int64_t)T * C * CG, "gconv: w [T][C][CG]");
  int ty[kMaxTaps], tx[kMaxTaps];
  for (int t = 0; t < T; ++t) { ty[t] = dy[t]; tx[t] = dx[t]; }
  const int rc = gconv_dgrad(bf(g), f32(w), bf(dxo), dxo.size(0), dxo.size(1), dxo.size(2), g.size(1), g.size(2), C, CG,
                             stride, T, ty, tx, cur_stream());
  TORCH_CHECK(rc == 0, "gconv_dgrad: no instantiation");
}

// x: the source map (fwd: x [N, IH, IW, C]; trans: dY [N, OH, OW, C]), y: the output map
void gconv_mfma_t(const at::Tensor& x, const at::Tensor& wpk, const at::Tensor& y, int64_t KW, int64_t stride,
                  bool trans, std::vector<int64_t> dy, std::vector<int64_t> dx) {
  CHECK_BF16(x); CHECK_BF16(y); CHECK_BF16(wpk);
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4 && x.size(0) == y.size(0) && x.size(3) == y.size(3), "gconv_mfma: NHWC maps");
  const int C = x.size(3), T = dy.size();
  TORCH_CHECK(C % 16 == 0 && T == 9 && dx.size() == dy.size() && (KW == 16 || KW == 32 || KW == 64), "gconv_mfma: C % 16, 3x3, KW");
  const int64_t nst = (9 * KW + 31) / 32;
  TORCH_CHECK(wpk.numel() == (int64_t)(C / 16) * nst * 64 * 8, "gconv_mfma: wpk [C/16][nst][64][8]");
  const at::Tensor& xi = trans ? y : x;   // input-space map
  const at::Tensor& yo = trans ? x : y;   // output-space map
  // shape contract the kernel indexes with: output-space size from the taps / stride (host-checked)
  int lo_y = 0, hi_y = 0, lo_x = 0, hi_x = 0;
  for (int t = 0; t < T; ++t) { lo_y = std::min(lo_y, (int)dy[t]); hi_y = std::max(hi_y, (int)dy[t]);
                                lo_x = std::min(lo_x, (int)dx[t]); hi_x = std::max(hi_x, (int)dx[t]); }
  TORCH_CHECK(yo.size(1) == (xi.size(1) - lo_y - hi_y - 1) / stride + 1 &&
              yo.size(2) == (xi.size(2) - lo_x - hi_x - 1) / stride + 1,
              "gconv_mfma: output size does not match the taps / stride");
  int ty[kMaxTaps], tx[kMaxTaps];
  for (int t = 0; t < T; ++t) { ty[t] = dy[t]; tx[t] = dx[t]; }
  const int rc = gconv_mfma(bf(x), bf(wpk), bf(y), xi.size(0), xi.size(1), xi.size(2), yo.size(1), yo.size(2), C,
                            (int)KW, (int)stride, trans, T, ty, tx, cur_stream());
  TORCH_CHECK(rc == 0, "gconv_mfma: no instantiation");
}

int64_t gconv_wgrad_mfma_slices_t(int64_t P, int64_t C) { return gconv_wgrad_mfma_slices(P, C); }

void gconv_wgrad_mfma_t(const at::Tensor& x, const at::Tensor& g, const at::Tensor& part, int64_t KW, int64_t stride,
                        std::vector<int64_t> dy, std::vector<int64_t> dx) {
  CHECK_BF16(x); CHECK_BF16(g); CHECK_F32(part);
  TORCH_CHECK(x.dim() == 4 && g.dim() == 4 && x.size(0) == g.size(0) && x.size(3) == g.size(3), "gconv_wgrad_mfma: NHWC maps");
  const int C = x.size(3), T = dy.size();
  TORCH_CHECK(C % 16 == 0 && T == 9 && dx.size() == dy.size() && (KW == 16 || KW == 32 || KW == 64), "gconv_wgrad_mfma: C % 16, 3x3, KW");
  const int64_t row = (int64_t)(C / 16) * (9 * KW / 16) * 256;
  TORCH_CHECK(part.numel() % row == 0 && part.numel() / row >= 1, "gconv_wgrad_mfma: part [S][C/16][9*KW/16][256]");
  int lo_y = 0, hi_y = 0, lo_x = 0, hi_x = 0;
  for (int t = 0; t < T; ++t) { lo_y = std::min(lo_y, (int)dy[t]); hi_y = std::max(hi_y, (int)dy[t]);
                                lo_x = std::min(lo_x, (int)dx[t]); hi_x = std::max(hi_x, (int)dx[t]); }
  TORCH_CHECK(g.size(1) == (x.size(1) - lo_y - hi_y - 1) / stride + 1 && g.size(2) == (x.size(2) - lo_x - hi_x - 1) / stride + 1,
              "gconv_wgrad_mfma: dY size does not match the taps / stride");
  int ty[kMaxTaps], tx[kMaxTaps];
  for (int t = 0; t < T; ++t) { ty[t] = dy[t]; tx[t] = dx[t]; }
  const int rc = gconv_wgrad_mfma(bf(x), bf(g), f32(part), (int)(part.numel() / row), x.size(0), x.size(1), x.size(2),
                                  g.size(1), g.size(2), C, (int)KW, (int)stride, T, ty, tx, cur_stream());
  TORCH_CHECK(rc == 0, "gconv_wgrad_mfma: no instantiation");
}

int64_t gconv_wgrad_slices_t(int64_t P, int64_t C, int64_t CG, int64_t T) { return gconv_wgrad_slices(P, C, CG, T); }

void gconv_wgrad_t(const at::Tensor& x, const at::Tensor& g, const at::Tensor& part, int64_t CG, int64_t stride,
                   std::vector<int64_t> dy, std::vector<int64_t> dx) {
  gconv_check(x, g, CG, dy, dx);
  CHECK_F32(part);
  const int C = x.size(3), T = dy.size();
  const int64_t nib = CG >= 8 ? CG / 8 : 1;
  const int64_t row = (int64_t)T * (C / 8) * nib * 64;
  TORCH_CHECK(part.numel() % row == 0, "gconv_wgrad: part [S][T*C/8*nib][64]");
  int ty[kMaxTaps], tx[kMaxTaps];
  for (int t = 0; t < T; ++t) { ty[t] = dy[t]; tx[t] = dx[t]; }
  const int rc = gconv_wgrad(bf(x), bf(g), f32(part), (int)(part.numel() / row), x.size(0), x.size(1), x.size(2),
                             g.size(1), g.size(2), C, CG, stride, T, ty, tx, cur_stream());
  TORCH_CHECK(rc == 0, "gconv_wgrad: no instantiation");
}

void colsum_t(const at::Tensor& part, const at::Tensor& out, bool accum) {
  CHECK_F32(part); CHECK_F32(out);
  const int64_t ncol = out.numel();
  TORCH_CHECK(part.numel() % ncol == 0, "colsum: part [nrow][ncol]");
  colsum(f32(part), part.numel() / ncol, ncol, f32(out), accum ? 1 : 0, cur_stream());
}
// ---- comm.hip: IPC peer-memory all-reduce -------------------------------------------------------
py::tuple comm_alloc_t(int64_t bytes) {
  void* p = nullptr;
  char h[kCommHandleBytes] = {0};
  const int rc = comm_alloc(bytes, &p, h);
  TORCH_CHECK(rc == 0, "comm_alloc: uncached allocation / IPC export failed (step ", rc, ")");
  return py::make_tuple(reinterpret_cast<int64_t>(p), py::bytes(h, kCommHandleBytes));
}

int64_t comm_open_t(py::bytes handle) {
  std::string h = handle;
  TORCH_CHECK((int)h.size() == kCommHandleBytes, "comm_open: bad IPC handle");
  void* p = nullptr;
  TORCH_CHECK(comm_open(h.data(), &p) == 0, "comm_open: hipIpcOpenMemHandle failed");
  return reinterpret_cast<int64_t>(p);
}

// in/out: fp64 rows (out may alias in); peers: every rank's mapped exchange buffer (own one included);
// epoch: int64 device counter (advanced by the kernel); err: int32 device error counter
void comm_allreduce_t(const at::Tensor& in, const at::Tensor& out, const std::vector<int64_t>& peers, int64_t rank,
                      int64_t cap, const at::Tensor& epoch, const at::Tensor& err, double timeout_s) {
  CHECK_DEV(in); CHECK_DEV(out); CHECK_I64(epoch); CHECK_DEV(err);
  TORCH_CHECK(in.scalar_type() == at::kDouble && out.scalar_type() == at::kDouble, "comm_allreduce: fp64 rows");
  TORCH_CHECK(err.scalar_type() == at::kInt && err.numel() >= 1 && epoch.numel() >= 1 && epoch.is_contiguous(),
              "comm_allreduce: state");
  const int world = (int)peers.size();
  TORCH_CHECK(world >= 1 && world <= kCommMaxRanks && rank >= 0 && rank < world, "comm_allreduce: bad rank/world");
  TORCH_CHECK(in.numel() == out.numel() && in.numel() <= cap, "comm_allreduce: ", in.numel(),
              " values exceed the exchange capacity ", cap);
  CommPeers pt{};
  for (int i = 0; i < world; ++i) {
    TORCH_CHECK(peers[i] != 0, "comm_allreduce: unmapped peer buffer");
    pt.buf[i] = reinterpret_cast<char*>(peers[i]);
  }
  int dev = 0, khz = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
  const long long ticks = (long long)(timeout_s * (khz > 0 ? khz : 100000) * 1000.0);
  oneshot_allreduce(in.data_ptr<double>(), out.data_ptr<double>(), in.numel(), pt, (int)rank, world, cap,
                    reinterpret_cast<unsigned long long*>(epoch.data_ptr<int64_t>()), (int)epoch.numel(),
                    err.data_ptr<int>(), ticks, cur_stream());
}

// ---- conv_bwd.hip: fused data- + weight-gradient of a narrow stride-1 conv ---------------------------
// ---- MAnet position attention (csrc/attention.hip) -----------------------------------------------------------
void batched_gemm_t(const at::Tensor& A, const at::Tensor& B, const at::Tensor& C, int64_t batch, int64_t M, int64_t N,
                    int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int64_t sa, int64_t sb, int64_t sc, bool ta, bool tb) {
  CHECK_BF16(A);
  CHECK_BF16(B);
  CHECK_DEV(C);
  const bool out_bf16 = C.scalar_type() == at::kBFloat16;
  TORCH_CHECK(out_bf16 || C.scalar_type() == at::kFloat, "C must be bf16 or fp32");
  // extent checks: the last element each operand's indexing can reach
  const int64_t a_last = (batch - 1) * sa + (ta ? (K - 1) * lda + M - 1 : (M - 1) * lda + K - 1);
  const int64_t b_last = (batch - 1) * sb + (tb ? (N - 1) * ldb + K - 1 : (K - 1) * ldb + N - 1);
  const int64_t c_last = (batch - 1) * sc + (M - 1) * ldc + N - 1;
  TORCH_CHECK(A.is_contiguous() && B.is_contiguous() && C.is_contiguous(), "contiguous operands");
  TORCH_CHECK(a_last < A.numel() && b_last < B.numel() && c_last < C.numel(), "batched_gemm: operand extents");
  const int rc = batched_gemm(bf(A), bf(B), C.data_ptr(), out_bf16, (int)batch, (int)M, (int)N, (int)K, (int)lda,
                              (int)ldb, (int)ldc, sa, sb, sc, ta, tb, cur_stream());
  TORCH_CHECK(rc == 0, "batched_gemm: bad shape");
}

void softmax_all_t(const at::Tensor& S, const at::Tensor& P, int64_t batch, int64_t n) {
  CHECK_F32(S);
  CHECK_BF16(P);
  TORCH_CHECK(S.numel() == batch * n && P.numel() == batch * n, "softmax_all: [batch][n]");
  softmax_all(S.data_ptr<float>(), bf(P), (int)batch, n, cur_stream());
}

void softmax_all_bwd_t(const at::Tensor& P, const at::Tensor& dP, const at::Tensor& dS, int64_t batch, int64_t n) {
  CHECK_BF16(P);
  CHECK_F32(dP);
  CHECK_BF16(dS);
  TORCH_CHECK(P.numel() == batch * n && dP.numel() == batch * n && dS.numel() == batch * n, "softmax_all_bwd: [batch][n]");
  softmax_all_bwd(bf(P), dP.data_ptr<float>(), bf(dS), (int)batch, n, cur_stream());
}

int64_t conv_bwd_fused_blocks_t(std::vector<int64_t> dims, std::vector<int64_t> dy, std::vector<int64_t> dx) {
  return conv_bwd_fused_blocks(make_geom(dims, dy, dx));
}

void conv_bwd_fused_t(const at::Tensor& dz, const c10::optional<at::Tensor>& gy, const c10::optional<at::Tensor>& gs,
                      const c10::optional<at::Tensor>& gk, bool grelu, const at::Tensor& x,
                      const c10::optional<at::Tensor>& xc, bool xrelu, const at::Tensor& wd, int64_t Kp_d,
                      const at::Tensor& dxo, const c10::optional<at::Tensor>& bn_y,
                      const c10::optional<at::Tensor>& bn_coef, bool bn_relu,
                      const c10::optional<at::Tensor>& stat_part, const at::Tensor& dw, std::vector<int64_t> dims,
                      std::vector<int64_t> dy, std::vector<int64_t> dx, const c10::optional<at::Tensor>& dz2,
                      const c10::optional<at::Tensor>& gy2, const c10::optional<at::Tensor>& gs2,
                      const c10::optional<at::Tensor>& gk2, bool grelu2, int64_t t1, bool accumulate) {
  ConvGeom g = make_geom(dims, dy, dx);
  const int64_t nblk = conv_bwd_fused_blocks(g);
  TORCH_CHECK(nblk > 0, "conv_bwd_fused: shape not eligible");
  const int64_t ny = (int64_t)g.N * g.OH * g.OW * g.Cgo, nx = (int64_t)g.N * g.IH * g.IW * g.Cgi;
  CHECK_BF16(dz); TORCH_CHECK(dz.numel() == ny, "dz numel");
  CHECK_BF16(x); TORCH_CHECK(x.numel() == nx, "x numel");
  CHECK_BF16(dxo); TORCH_CHECK(dxo.numel() == nx, "dx numel");
  CHECK_BF16(wd);
  TORCH_CHECK(Kp_d % 32 == 0 && Kp_d >= g.T * g.Go * g.Cgo && wd.numel() >= 32 * Kp_d, "packed dgrad weights");
  CHECK_F32(dw); TORCH_CHECK(dw.numel() == nblk * g.Go * g.Cgo * g.T * g.Cgi, "dw slabs numel");
  FusedBwdArgs a{};
  a.dz = bf(dz);
  a.t1 = (int)t1;
  if (g.Go == 2) {
    TORCH_CHECK(dz2.has_value() && dz2->defined(), "conv_bwd_fused: Go == 2 needs dz2");
    CHECK_BF16(*dz2); TORCH_CHECK(dz2->numel() == ny, "dz2 numel");
    a.dz2 = bf(*dz2);
    if (gy2.has_value() && gy2->defined()) {
      CHECK_BF16(*gy2); TORCH_CHECK(gy2->numel() == ny, "gy2 numel");
      TORCH_CHECK(gs2.has_value() && gk2.has_value(), "gy2 needs gs2 and gk2");
      CHECK_F32(*gs2); CHECK_F32(*gk2);
      TORCH_CHECK(gs2->numel() >= 2 * g.Cgo && gk2->numel() >= 3 * g.Cgo, "gs2 [4][C], gk2 [3][C]");
      a.gy2 = bf(*gy2); a.gs2 = gs2->data_ptr<float>(); a.gk2 = gk2->data_ptr<float>();
    }
    a.grelu2 = grelu2 ? 1 : 0;
  }
  if (gy.has_value() && gy->defined()) {
    CHECK_BF16(*gy); TORCH_CHECK(gy->numel() == ny, "gy numel");
    TORCH_CHECK(gs.has_value() && gk.has_value(), "gy needs gs and gk");
    CHECK_F32(*gs); CHECK_F32(*gk);
    TORCH_CHECK(gs->numel() >= 2 * g.Cgo && gk->numel() >= 3 * g.Cgo, "gs [4][C], gk [3][C]");
    a.gy = bf(*gy); a.gs = gs->data_ptr<float>(); a.gk = gk->data_ptr<float>();
  }
  a.grelu = grelu ? 1 : 0;
  a.x = bf(x);
  a.xc = f32_opt(xc);
  if (a.xc) TORCH_CHECK(xc->numel() >= 2 * g.Cgi, "xc [4][C]");
  a.xrelu = xrelu ? 1 : 0;
  a.wd = bf(wd);
  a.Kp = (int)Kp_d;
  a.dxo = bf(dxo);
  if (bn_y.has_value() && bn_y->defined()) {
    CHECK_BF16(*bn_y); TORCH_CHECK(bn_y->numel() == nx, "bn_y numel");
    TORCH_CHECK(bn_coef.has_value() && stat_part.has_value(), "BN epilogue needs bn_coef and stat_part");
    CHECK_F32(*bn_coef); CHECK_F32(*stat_part);
    TORCH_CHECK(bn_coef->numel() >= 3 * g.Cgi && stat_part->numel() == nblk * 2 * g.Cgi, "BN epilogue shapes");
    a.bn_y = bf(*bn_y); a.bn_coef = bn_coef->data_ptr<float>(); a.stat_part = stat_part->data_ptr<float>();
  }
  a.bn_relu = bn_relu ? 1 : 0;
  a.dw = f32(dw);
  a.accum = accumulate ? 1 : 0;
  const int rc = conv_bwd_fused(a, g, cur_stream());
  TORCH_CHECK(rc == 0, "conv_bwd_fused: launch failed (", rc, ")");
}

}  // namespace

extern "C" const char* msp_sources_sha();   // build/csrc/sources_sha.cpp (generated by csrc/build.py)

PYBIND11_MODULE(_C, m) {
  m.doc() = "MI355X (gfx950) HIP kernels for medical_segmentation_pytorch_amd";
  m.def("conv_fwd", &conv_fwd, py::arg("xs"), py::arg("wp"), py::arg("ys"), py::arg("bias"), py::arg("stat_part"),
        py::arg("dims"), py::arg("dy"), py::arg("dx"), py::arg("trans"), py::arg("xc") = OptTensors{},
        py::arg("xrelu") = 0, py::arg("accumulate") = false, py::arg("gy") = OptTensors{},
        py::arg("gs") = OptTensors{}, py::arg("gk") = OptTensors{}, py::arg("grelu") = 0);
  m.def("conv_fwd_bn", &conv_fwd_bn, py::arg("xs"), py::arg("wp"), py::arg("ys"), py::arg("stat_part"), py::arg("dims"),
        py::arg("dy"), py::arg("dx"), py::arg("bn_y"), py::arg("bn_coef"), py::arg("relu"), py::arg("gy") = OptTensors{},
        py::arg("gs") = OptTensors{}, py::arg("gk") = OptTensors{}, py::arg("grelu") = 0);
  m.def("conv_wgrad", &conv_wgrad_t, py::arg("dys"), py::arg("xs"), py::arg("dw"), py::arg("dims"), py::arg("dy"),
        py::arg("dx"), py::arg("trans"), py::arg("xc") = OptTensors{}, py::arg("xrelu") = 0,
        py::arg("gy") = OptTensors{}, py::arg("gs") = OptTensors{}, py::arg("gk") = OptTensors{}, py::arg("grelu") = 0);
  m.def("conv_wgrad_uses_halo", &conv_wgrad_uses_halo_t);
  m.def("conv_pick_mi", &conv_pick_mi);
  m.def("conv_rows_alloc", &conv_rows_alloc);
  m.def("conv_stat_blocks", &conv_stat_blocks_t, py::arg("dims"), py::arg("dy"), py::arg("dx"), py::arg("trans") = false,
        py::arg("bwd") = false, py::arg("bne") = false);
  m.def("conv_uses_halo", &conv_uses_halo_t, py::arg("dims"), py::arg("dy"), py::arg("dx"), py::arg("trans"),
        py::arg("bwd") = false);
  m.def("conv_set_halo", [](bool on) { conv_set_halo(on ? 1 : 0); });
  m.def("conv_set_halo_split", [](int64_t mode) { conv_set_halo_split((int)mode); });
  m.def("conv_set_gemm", [](bool on) { conv_gemm_set(on ? 1 : 0); });
  m.def("conv_gemm_force_cfg", [](int64_t c) { conv_gemm_force_cfg((int)c); });
  m.def("conv_gemm_num_cfgs", []() { return conv_gemm_num_cfgs(); });
  m.def("conv_set_wgrad_gemm", [](int64_t mode) { conv_wgrad_gemm_set((int)mode); });
  m.def("conv_wgrad_gemm_force_cfg", [](int64_t c) { conv_wgrad_gemm_force_cfg((int)c); });
  m.def("conv_wgrad_gemm_num_cfgs", []() { return conv_wgrad_gemm_num_cfgs(); });
  m.def("conv_uses_wgrad_gemm", [](std::vector<int64_t> dims, std::vector<int64_t> dy, std::vector<int64_t> dx, bool trans) {
    return conv_wgrad_gemm_ok(make_geom(dims, dy, dx), trans);
  });
  m.def("conv_uses_gemm", [](std::vector<int64_t> dims, std::vector<int64_t> dy, std::vector<int64_t> dx, bool trans) {
    return conv_gemm_ok(make_geom(dims, dy, dx), trans);
  });
  m.def("conv_set_phase", [](bool on) { conv_set_phase(on ? 1 : 0); });
  m.def("pack_weight", &pack_weight_t);
  m.def("unpack_wgrad", &unpack_wgrad_t, py::arg("src"), py::arg("dst"), py::arg("nrow"), py::arg("nch"),
        py::arg("T"), py::arg("Cpk"), py::arg("Ktot"), py::arg("t_base"), py::arg("c_base"), py::arg("s_row"),
        py::arg("s_ch"), py::arg("accumulate"), py::arg("nrep") = 1, py::arg("rep_stride") = 0);
  m.def("conv_wgrad_replicas", &conv_wgrad_replicas_t, py::arg("dims"), py::arg("dy"), py::arg("dx"), py::arg("trans"),
        py::arg("bwd") = false, py::arg("pro") = false);
  m.def("pack_batch", &pack_batch_t);
  m.def("pack_per_block", &pack_per_block);
  m.def("bn_partial_blocks", [](int64_t P, int64_t Cp) { return bn_partial_blocks(P, Cp); });
  m.def("sum_stats", &sum_stats_t, py::arg("inputs"), py::arg("out"), py::arg("part"), py::arg("P"), py::arg("Cp"),
        py::arg("coefs") = OptTensors{}, py::arg("relu_mask") = 0);
  m.def("bn_reduce_partials", &bn_reduce_partials_t);
  m.def("bn_reduce_splits", [](int64_t nblk) { return bn_reduce_splits(nblk); });
  m.def("bn_collapse", &bn_collapse_t);
  m.def("bn_finalize", &bn_finalize_t);
  m.def("bn_reduce_finalize", &bn_reduce_finalize_t);
  m.def("bn_reduce_bwd_finalize", &bn_reduce_bwd_finalize_t);
  m.def("bn_rf_chunks", [](int64_t Cp) { return bn_rf_chunks((int)Cp); });
  m.def("bn_act_apply", &bn_act_apply_t);
  m.def("bn_act_apply_relu6", &bn_act_apply_relu6_t);
  m.def("bn_add_act", &bn_add_act_t);
  m.def("gconv_fwd", &gconv_fwd_t);
  m.def("relu6", &relu6_t);
  m.def("relu6_bwd", &relu6_bwd_t);
  m.def("bn_aug_mask", &bn_aug_mask_t);
  m.def("gconv_dgrad", &gconv_dgrad_t);
  m.def("gconv_wgrad_slices", &gconv_wgrad_slices_t);
  m.def("gconv_wgrad", &gconv_wgrad_t);
  m.def("gconv_mfma", &gconv_mfma_t);
  m.def("gconv_wgrad_mfma", &gconv_wgrad_mfma_t);
  m.def("gconv_wgrad_mfma_slices", &gconv_wgrad_mfma_slices_t);
  m.def("aug_gray_scratch_doubles", &aug_gray_scratch_doubles);
  m.def("bn_act_bwd_partial", &bn_act_bwd_partial_t);
  m.def("bn_bwd_finalize", &bn_bwd_finalize_t, py::arg("tmp"), py::arg("C"), py::arg("Cp"), py::arg("count"),
        py::arg("stats"), py::arg("dgamma"), py::arg("dbeta"), py::arg("coef"), py::arg("pscale") = 1.0);
  m.def("bn_act_bwd_apply", &bn_act_bwd_apply_t);
  m.def("bn_act_bwd_apply_part", &bn_act_bwd_apply_part_t);
  m.def("bn_tail_partial", &bn_tail_partial_t);
  m.def("bn_tail_apply", &bn_tail_apply_t, py::arg("dz"), py::arg("ys"), py::arg("ostats"), py::arg("ocoef"),
        py::arg("orelu"), py::arg("y"), py::arg("st"), py::arg("coef"), py::arg("relu_mask"), py::arg("dy"),
        py::arg("P"), py::arg("Cp"), py::arg("g") = py::none());
  m.def("bn_tail_blocks", [](int64_t P, int64_t Cp) { return bn_tail_blocks(P, (int)Cp); });
  m.attr("kTailMax") = kTailMax;
  m.attr("kTailMaxCp") = kTailMaxCp;
  m.def("nchw_to_nhwc", &nchw_to_nhwc_t);
  m.def("nhwc_to_nchw", &nhwc_to_nchw_t);
  m.def("up2_add", &up2_add_t, py::arg("low"), py::arg("skip"), py::arg("out"), py::arg("N"), py::arg("h"),
        py::arg("w"), py::arg("Cp"), py::arg("coefs") = OptTensors{}, py::arg("relu_mask") = 0);
  m.def("pool2_sum", &pool2_sum_t);
  m.def("add_n", &add_n_t, py::arg("inputs"), py::arg("out"), py::arg("coefs") = OptTensors{},
        py::arg("relu_mask") = 0);
  m.def("scale_f32", &scale_f32_t);
  m.def("aug_batch", &aug_batch_t);
  m.def("bilinear_resize", &bilinear_resize_t);
  m.def("colorize", &colorize_t);
  m.def("aug_iparams", []() { return kAugIParams; });
  m.def("maxpool_fwd", &maxpool_fwd_t);
  m.def("maxpool_bwd", &maxpool_bwd_t);
  m.def("up2_cat", &up2_cat_t);
  m.def("up2_cat_bwd", &up2_cat_bwd_t);
  m.def("add_act", &add_act_t);
  m.def("relu_bwd", &relu_bwd_t);
  m.def("ce_blocks", &ce_blocks_t);
  m.def("ce_fwd_bwd", &ce_fwd_bwd_t);
  m.def("kd_kl_fwd_bwd", &kd_kl_fwd_bwd_t);
  m.def("ohem_select", &ohem_select_t);
  m.def("ohem_backward", &ohem_backward_t);
  m.def("ohem_state_words", []() { return ohem_state_words(); });
  m.def("mse_fwd_bwd", &mse_fwd_bwd_t);
  m.def("bce_dice_stats", &bce_dice_stats_t);
  m.def("bce_dice_grad", &bce_dice_grad_t);
  m.def("bce_dice_splits", &bce_dice_splits_t);
  m.def("adam_step", &adam_step_t, py::arg("p"), py::arg("g"), py::arg("m"), py::arg("v"), py::arg("hyper"),
        py::arg("adamw"), py::arg("amp") = py::none());
  m.def("sgd_step", &sgd_step_t, py::arg("p"), py::arg("g"), py::arg("buf"), py::arg("hyper"),
        py::arg("amp") = py::none());
  m.def("amp_check", &amp_check_t);
  m.def("amp_update", &amp_update_t);
  m.def("ema_update", &ema_update_t);
  m.def("confmat_update", &confmat_update_t);
  m.def("resize_bilinear", &resize_bilinear_t, py::arg("x"), py::arg("y"), py::arg("sh"), py::arg("sw"),
        py::arg("align"), py::arg("accum") = false, py::arg("backward") = false);
  m.def("nc_sums_blocks", &nc_sums_blocks_t);
  m.def("nc_sums", &nc_sums_t, py::arg("x"), py::arg("dz"), py::arg("tab"), py::arg("relu"), py::arg("part"));
  m.def("gn_finalize", &gn_finalize_t);
  m.def("gn_bwd_finalize", &gn_bwd_finalize_t);
  m.def("affine_nc", &affine_nc_t);
  m.def("affine_nc_bwd", &affine_nc_bwd_t);
  m.def("adaptive_avgpool", &adaptive_avgpool_t, py::arg("x"), py::arg("y"), py::arg("backward") = false);
  m.def("dwconv_fwd", &dwconv_fwd_t);
  m.def("dwconv_wgrad_blocks", &dwconv_wgrad_blocks_t);
  m.def("dwconv_wgrad", &dwconv_wgrad_t);
  m.def("colsum", &colsum_t);
  m.def("conv_bwd_fused_blocks", &conv_bwd_fused_blocks_t);
  m.def("batched_gemm", &batched_gemm_t);
  m.def("softmax_all", &softmax_all_t);
  m.def("softmax_all_bwd", &softmax_all_bwd_t);
  m.def("conv_set_fwd_fused", [](int64_t mode) { conv_set_fwd_fused((int)mode); });   // 0 / 1 / 2 (see conv_bwd.hip)
  m.def("conv_fwd_fused_ok", [](std::vector<int64_t> dims, std::vector<int64_t> dy, std::vector<int64_t> dx) {
    return conv_fwd_fused_ok(make_geom(dims, dy, dx));
  });
  m.def("conv_bwd_fused", &conv_bwd_fused_t, py::arg("dz"), py::arg("gy"), py::arg("gs"), py::arg("gk"),
        py::arg("grelu"), py::arg("x"), py::arg("xc"), py::arg("xrelu"), py::arg("wd"), py::arg("Kp_d"), py::arg("dxo"),
        py::arg("bn_y"), py::arg("bn_coef"), py::arg("bn_relu"), py::arg("stat_part"), py::arg("dw"), py::arg("dims"),
        py::arg("dy"), py::arg("dx"), py::arg("dz2") = py::none(), py::arg("gy2") = py::none(),
        py::arg("gs2") = py::none(), py::arg("gk2") = py::none(), py::arg("grelu2") = false, py::arg("t1") = -1,
        py::arg("accumulate") = false);
  m.def("comm_buffer_bytes", &comm_buffer_bytes);
  m.def("comm_alloc", &comm_alloc_t);
  m.def("comm_open", &comm_open_t);
  m.def("comm_close", [](int64_t p) { comm_close(reinterpret_cast<void*>(p)); });
  m.def("comm_free", [](int64_t p) { comm_free(reinterpret_cast<void*>(p)); });
  m.def("comm_allreduce", &comm_allreduce_t);
  m.def("comm_max_ranks", []() { return kCommMaxRanks; });
  m.def("sources_sha", []() { return std::string(msp_sources_sha()); });
  m.def("comm_wall_clock_khz", []() {
    int dev = 0, khz = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
    return (int64_t)(khz > 0 ? khz : 100000);
  });
}
