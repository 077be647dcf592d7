"""One-off source patch (kept for the record): halo wgrad with NCB 32-row dY sub-tiles per block sharing
one staged input halo, plus the StagedScalars host->device race fix."""
ROOT = '/root/repo/'


def sub(path, old, new, count=1):
    p = ROOT + path
    s = open(p).read()
    assert s.count(old) >= 1, (path, old[:80])
    s = s.replace(old, new, count)
    open(p, 'w').write(s)


# ---------------------------------------------------------------- conv.hip: wgrad halo kernel
p = ROOT + 'csrc/conv.hip'
s = open(p).read()
start = s.index('constexpr int kDwWaves = 8;')
end = s.index('__global__ void pack_weight_kernel')
new_kernel = r'''constexpr int kDwWaves = 8;      // waves per block: each owns <= 3 (tap, ci16) pairs of a 3x3
constexpr int kDwMaxHalo = 640;  // halo pixels the staging registers cover (every T <= 9 tap set)
constexpr long kDwSplitTarget = 256;
constexpr int kDwMaxNcb = 3;     // 32-row dY sub-tiles per block, all sharing ONE staged input halo
constexpr int kDwMaxLds = 120 * 1024;
// staging elements per thread: NCB dY sub-tiles (2 slots of 128 pixels each) + the halo
constexpr int dw_stage(int ncb) { return 2 * ncb + kDwMaxHalo / (16 * kDwWaves); }

DEVI int dw_elem(int pix, int half, int sub4) {   // element offset of (pixel, 16-ch half, 4-ch sub)
  return pix * DW_CH + 16 * (half ^ ((pix >> 3) & 1)) + 4 * sub4;
}

// NCB > 1 (wide dY: horizontally fused convs, wide layers): the block owns NCB consecutive 32-row co
// sub-tiles.  The input halo is staged, and every B fragment read from LDS, ONCE per slice for all of
// them: one input pass per NCB sub-tiles instead of per sub-tile, and fewer LDS reads/writes per MFMA.
template <int NPW, int NCB>
__global__ __launch_bounds__(64 * kDwWaves) void conv_wgrad_halo_kernel(WgradPtrs P, float* __restrict__ dw, ConvGeom g,
                                                              DwTile tl, int KT, long ntiles, int nrep) {
  constexpr int NST = dw_stage(NCB);
  extern __shared__ __attribute__((aligned(16))) uint16_t dsm[];
  constexpr int NPX = 256, NSL = 8, SUB = NPX * DW_CH;
  uint16_t* sY = dsm;                       // [NCB][256][32]  swizzled
  uint16_t* sX = dsm + NCB * SUB;           // [HH * HWd][32]  swizzled
  __shared__ int2 s_tap[kMaxTaps];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4, q = lr >> 2, p4 = lr & 3;
  const int co0 = blockIdx.y * DW_CH * NCB, ci0 = blockIdx.z * DW_CH;
  const int rows = g.Go * g.Cgo, Cip = g.Gi * g.Cgi;
  if (tid < kMaxTaps) s_tap[tid] = make_int2(g.dy[tid] - tl.ey0, g.dx[tid] - tl.ex0);

  // per-thread loader roles: vector vv = tid & 3 (8 channels), pixel lane vp = tid >> 2 (16 per wave)
  const int vv = tid & 3, vp = tid >> 2;
  const uint16_t* y_base[NCB];
  bool y_ok[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    const int yco = co0 + DW_CH * cb + 8 * vv;
    y_ok[cb] = yco < rows;
    const int y_g = y_ok[cb] ? yco / g.Cgo : 0;
    y_base[cb] = P.dy[y_g] + (y_ok[cb] ? yco - y_g * g.Cgo : 0);
  }
  const int xci = ci0 + 8 * vv;
  const bool x_ok = xci < Cip;
  const int x_g = x_ok ? xci / g.Cgi : 0;
  const uint16_t* x_base = P.x[x_g] + (xci - x_g * g.Cgi);
  __syncthreads();

  // lane pixel within a 32-pixel slice: lo = 8*lg + q, hi = lo + 4 (tile coords: row ry, column cx)
  const int plo = 8 * lg + q, phi = plo + 4;
  const int ry_lo = plo >> tl.tw_shift, cx_lo = plo & (tl.TW - 1);
  const int ry_hi = phi >> tl.tw_shift, cx_hi = phi & (tl.TW - 1);
  const int rows_per_slice = 32 >> tl.tw_shift;
  // A (dY) read offsets: slice sl adds 32*32*sl (bit 3 of the pixel is lg & 1 for every slice)
  int offA[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) { offA[i][0] = dw_elem(plo, i, p4); offA[i][1] = dw_elem(phi, i, p4); }
  // B (halo) read offsets per owned (tap, ci16) pair: slice sl adds rows_per_slice*sl*HWd*32.
  // Only the 16-channel halves that hold real channels are paired (a 40-channel input's second chunk
  // has one), and co halves past `rows` are skipped: no MFMA runs on all-padding tiles.
  const int nhv = min(2, (Cip - ci0 + 15) >> 4);
  int nco[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) nco[cb] = max(0, min(2, (rows - co0 - DW_CH * cb + 15) >> 4));
  const int npairs = nhv * g.T;
  int offB[NPW][2];
#pragma unroll
  for (int j = 0; j < NPW; ++j) {
    const int pr = wave + kDwWaves * j;
    const int t = pr < npairs ? pr / nhv : 0, cf = pr < npairs ? pr - t * nhv : 0;
    const int2 d = s_tap[t];
    offB[j][0] = dw_elem((ry_lo + d.x) * tl.HWd + cx_lo + d.y, cf, p4);
    offB[j][1] = dw_elem((ry_hi + d.x) * tl.HWd + cx_hi + d.y, cf, p4);
  }

  f32x4_t acc[NCB][2][NPW];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NPW; ++j) acc[cb][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nh = tl.HH * tl.HWv;
  // Software pipeline over the block's tiles: a tile's staging loads (NST x 16 B per thread,
  // host-checked) are issued into registers before the previous tile's MFMA phase and written to LDS
  // after it, so HBM latency hides under the MFMAs.  Slot u < 2*NCB is dY sub-tile u/2 (pixels
  // vp + 128*(u&1)); the other slots walk the halo.
  uint4 sv[NST];
  int sd[NST];
  auto stage_load = [&](long tix) {
    const int per_img = tl.tiles_y * tl.tiles_x;
    const int n = (int)(tix / per_img);
    const int rem = (int)(tix - (long)n * per_img);
    const int y0 = (rem / tl.tiles_x) * tl.TH, x0 = (rem % tl.tiles_x) * tl.TW;
    const long yoff = (long)n * g.OH * g.OW * g.Cgo;
    const uint16_t* xim = x_base + (long)n * g.IH * g.IW * g.Cgi;
#pragma unroll
    for (int u = 0; u < NST; ++u) {
      sv[u] = make_uint4(0, 0, 0, 0);
      sd[u] = -1;
      if (u < 2 * NCB) {
        const int cb = u >> 1, e = vp + 16 * kDwWaves * (u & 1);
        const int oy = y0 + (e >> tl.tw_shift), ox = x0 + (e & (tl.TW - 1));
        sd[u] = cb * SUB + dw_elem(e, vv >> 1, 2 * (vv & 1));
        if (y_ok[cb] && oy < g.OH && ox < g.OW)
          sv[u] = *reinterpret_cast<const uint4*>(y_base[cb] + yoff + (oy * g.OW + ox) * g.Cgo);
      } else {
        const int hp = vp + 16 * kDwWaves * (u - 2 * NCB);
        if (hp < nh) {
          const int hy = fdiv(hp, tl.HWv, tl.inv_hwv), hx = hp - __mul24(hy, tl.HWv);
          const int iy = y0 + hy + tl.ey0, ix = x0 + hx + tl.ex0;
          sd[u] = NCB * SUB + dw_elem(hy * tl.HWd + hx, vv >> 1, 2 * (vv & 1));
          if (x_ok && (unsigned)iy < (unsigned)g.IH && (unsigned)ix < (unsigned)g.IW)
            sv[u] = *reinterpret_cast<const uint4*>(xim + (iy * g.IW + ix) * g.Cgi);
        }
      }
    }
  };
  if ((long)blockIdx.x < ntiles) stage_load(blockIdx.x);
  for (long tix = blockIdx.x; tix < ntiles; tix += gridDim.x) {
    __syncthreads();   // previous tile's LDS reads are done
#pragma unroll
    for (int u = 0; u < NST; ++u)
      if (sd[u] >= 0) *reinterpret_cast<uint4*>(&sY[sd[u]]) = sv[u];
    __syncthreads();
    if (tix + gridDim.x < ntiles) stage_load(tix + gridDim.x);   // in flight during the MFMAs
    for (int sl = 0; sl < NSL; ++sl) {
      const int sa = sl * 32 * DW_CH, sb = sl * rows_per_slice * tl.HWd * DW_CH;
      uint4 fa[NCB][2];
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          fa[cb][i] = make_uint4(0, 0, 0, 0);
          if (i < nco[cb]) {   // block-uniform: EXEC stays all ones for the transposed reads
            const uint2 lo = tr_read(&sY[cb * SUB + sa + offA[i][0]]);
            const uint2 hi = tr_read(&sY[cb * SUB + sa + offA[i][1]]);
            fa[cb][i] = make_uint4(lo.x, lo.y, hi.x, hi.y);
          }
        }
#pragma unroll
      for (int j = 0; j < NPW; ++j) {
        if (wave + kDwWaves * j < npairs) {
          const uint2 lo = tr_read(&sX[sb + offB[j][0]]);
          const uint2 hi = tr_read(&sX[sb + offB[j][1]]);
          const uint4 fb = make_uint4(lo.x, lo.y, hi.x, hi.y);
#pragma unroll
          for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
            for (int i = 0; i < 2; ++i)
              if (i < nco[cb]) acc[cb][i][j] = mfma16x16x32(fa[cb][i], fb, acc[cb][i][j]);
        }
      }
    }
  }
  // every block adds into one of nrep dW replicas (summed by unpack_wgrad): spreads the adds of
  // ~nsplit blocks over nrep x more addresses instead of hot-spotting a few L2 lines
  float* dwr = dw + (long)(blockIdx.x % nrep) * rows * KT;
#pragma unroll
  for (int j = 0; j < NPW; ++j) {
    const int pr = wave + kDwWaves * j;
    if (pr >= npairs) continue;
    const int t = pr / nhv, cf = pr - t * nhv;
    const int ci = ci0 + 16 * cf + lr;
    if (ci >= Cip) continue;
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = co0 + DW_CH * cb + 16 * i + 4 * lg + r;
          if (co < rows && (co % g.Cgo) < g.Cgo_l) atomicAdd(&dwr[(long)co * KT + t * Cip + ci], acc[cb][i][j][r]);
        }
  }
}

'''
s = s[:start] + new_kernel + s[end:]
assert s.count('DEVI int dw_elem') == 1

# host side
old = '''static size_t wgrad_halo_lds(const DwTile& tl) { return ((size_t)256 + (size_t)tl.HH * tl.HWd) * DW_CH * 2; }'''
assert old in s
s = s.replace(old, '''static size_t wgrad_halo_lds(const DwTile& tl, int ncb) {
  return ((size_t)256 * ncb + (size_t)tl.HH * tl.HWd) * DW_CH * 2;
}''')
old = '''  if (256 + tl.HH * tl.HWv > 16 * kDwWaves * kDwStage) return false;   // the pipelined staging registers
  return wgrad_halo_lds(tl) <= 64 * 1024;'''
assert old in s
s = s.replace(old, '''  if (tl.HH * tl.HWv > kDwMaxHalo) return false;   // the pipelined staging registers
  return wgrad_halo_lds(tl, 1) <= 64 * 1024;''')
old = '''    const long ntiles = (long)g.N * tl.tiles_y * tl.tiles_x;
    const int gy = cdiv(rows, DW_CH), gz = cdiv(g.Gi * g.Cgi, DW_CH);'''
assert old in s
s = s.replace(old, '''    const long ntiles = (long)g.N * tl.tiles_y * tl.tiles_x;
    // co sub-tiles per block: as many as the LDS budget allows (<= kDwMaxNcb; env MSP_DW_NCB caps it)
    static int max_ncb = -1;
    if (max_ncb < 0) {
      const char* e = getenv("MSP_DW_NCB");
      max_ncb = (e != nullptr && atoi(e) > 0) ? std::min(atoi(e), kDwMaxNcb) : kDwMaxNcb;
    }
    int ncb = std::min(max_ncb, cdiv(rows, DW_CH));
    while (ncb > 1 && wgrad_halo_lds(tl, ncb) > (size_t)kDwMaxLds) --ncb;
    const int gy = cdiv(rows, DW_CH * ncb), gz = cdiv(g.Gi * g.Cgi, DW_CH);''')
old = '''    const size_t lds = wgrad_halo_lds(tl);
    dim3 grid((unsigned)nsplit, gy, gz);
    const int npw = cdiv(2 * g.T, kDwWaves);
#define HW_(N_) if (npw == N_) { hipLaunchKernelGGL((conv_wgrad_halo_kernel<N_>), grid, dim3(64 * kDwWaves), lds, s, P, dw, g, tl, KT, ntiles, nrep); return; }
    HW_(1) HW_(2) HW_(3)
#undef HW_'''
assert old in s
s = s.replace(old, '''    const size_t lds = wgrad_halo_lds(tl, ncb);
    dim3 grid((unsigned)nsplit, gy, gz);
    const int npw = cdiv(2 * g.T, kDwWaves);
    // > 64 KB of dynamic LDS (gfx950 has 160 KB per CU) is opted into once per instantiation, before any
    // graph capture (the first call of every shape runs eagerly)
#define HW_(N_, C_)                                                                                      \\
    if (npw == N_ && ncb == C_) {                                                                       \\
      static bool lds_attr = false;                                                                     \\
      if (!lds_attr) {                                                                                  \\
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_wgrad_halo_kernel<N_, C_>),       \\
                                  hipFuncAttributeMaxDynamicSharedMemorySize, kDwMaxLds);               \\
        lds_attr = true;                                                                                \\
      }                                                                                                 \\
      hipLaunchKernelGGL((conv_wgrad_halo_kernel<N_, C_>), grid, dim3(64 * kDwWaves), lds, s, P, dw, g, tl, KT, \\
                         ntiles, nrep);                                                                 \\
      return;                                                                                           \\
    }
    HW_(1, 1) HW_(2, 1) HW_(3, 1) HW_(1, 2) HW_(2, 2) HW_(3, 2) HW_(1, 3) HW_(2, 3) HW_(3, 3)
#undef HW_''')
assert 'kDwStage' not in s, 'stale kDwStage reference'
open(p, 'w').write(s)

# ---------------------------------------------------------------- StagedScalars race fix
sub('medical_segmentation_pytorch_amd/runtime/engine.py', '''class FlatOptimizer:''', '''class StagedScalars:
    """A small device fp32 tensor refreshed from pinned host memory once per step, race-free.

    The host runs ahead of the GPU (hipGraph replays / eager launches are asynchronous), so a single
    pinned staging buffer could be overwritten with step k+1's values before the DMA of step k's
    copy has read it.  The staging buffers form a ring; a slot is rewritten only after the event
    recorded behind its previous copy completed (a stall only if the host is ``depth`` steps ahead).
    ``dev`` keeps its address, so graphs that captured it stay valid."""

    def __init__(self, n, device, depth=8):
        self.dev = torch.zeros(n, dtype=torch.float32, device=device)
        self.cuda = self.dev.is_cuda
        self.ring = [torch.zeros(n, dtype=torch.float32).pin_memory() if self.cuda else torch.zeros(n)
                     for _ in range(depth)]
        self.events = [None] * depth
        self.i = 0

    def host(self):
        """The next writable pinned buffer (waits for its previous copy if still in flight)."""
        ev = self.events[self.i]
        if ev is not None:
            ev.synchronize()
        return self.ring[self.i]

    def push(self):
        """Enqueue the H2D copy of the buffer returned by :meth:`host` on the current stream."""
        buf = self.ring[self.i]
        self.dev.copy_(buf, non_blocking=True)
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record()
            self.events[self.i] = ev
        self.i = (self.i + 1) % len(self.ring)


class FlatOptimizer:''')
sub('medical_segmentation_pytorch_amd/runtime/engine.py', '''        self.hyper = torch.zeros(8, dtype=torch.float32, device=dev)
        self.hyper_host = torch.zeros(8, dtype=torch.float32).pin_memory() if torch.cuda.is_available() \\
            else torch.zeros(8, dtype=torch.float32)
        self.grad_scale = 1.0''', '''        self.staged = StagedScalars(8, dev)
        self.hyper = self.staged.dev
        self.grad_scale = 1.0''')
sub('medical_segmentation_pytorch_amd/runtime/engine.py', '''        self.step_count += 1
        h = self.hyper_host''', '''        self.step_count += 1
        h = self.staged.host()''')
sub('medical_segmentation_pytorch_amd/runtime/engine.py', '''            h[0], h[1], h[2], h[3] = self.lr, self.momentum, self.wd, self.grad_scale
        self.hyper.copy_(h, non_blocking=True)''', '''            h[0], h[1], h[2], h[3] = self.lr, self.momentum, self.wd, self.grad_scale
        self.staged.push()''')
sub('medical_segmentation_pytorch_amd/utils/optimizer.py', '''        self.hyper = torch.zeros(8, dtype=torch.float32, device=device)
        self.hyper_host = torch.zeros(8, dtype=torch.float32)
        if device.type == 'cuda':
            self.hyper_host = self.hyper_host.pin_memory()
        self.bucketer = None''', '''        from ..runtime.engine import StagedScalars
        self.staged = StagedScalars(8, device)
        self.hyper = self.staged.dev
        self.bucketer = None''')
sub('medical_segmentation_pytorch_amd/utils/optimizer.py', '''        h = self.hyper_host''', '''        h = self.staged.host()''')
sub('medical_segmentation_pytorch_amd/utils/optimizer.py', '''            h[7] = self.grad_scale
        self.hyper.copy_(h, non_blocking=True)''', '''            h[7] = self.grad_scale
        self.staged.push()''')
sub('medical_segmentation_pytorch_amd/runtime/trainer_engine.py',
    '''from .engine import Arena, FlatOptimizer, GradBucketer, OneCycle, stat_group''',
    '''from .engine import Arena, FlatOptimizer, GradBucketer, OneCycle, StagedScalars, stat_group''')
sub('medical_segmentation_pytorch_amd/runtime/trainer_engine.py', '''        self.ema_hyper = torch.zeros(1, device=dev)
        self.ema_hyper_host = torch.zeros(1).pin_memory()''', '''        self.ema_staged = StagedScalars(1, dev)
        self.ema_hyper = self.ema_staged.dev''')
sub('medical_segmentation_pytorch_amd/runtime/trainer_engine.py', '''        self.ema_hyper_host[0] = d
        self.ema_hyper.copy_(self.ema_hyper_host, non_blocking=True)''', '''        self.ema_staged.host()[0] = d
        self.ema_staged.push()''')
for f in ('runtime/engine.py', 'utils/optimizer.py', 'runtime/trainer_engine.py'):
    assert 'hyper_host' not in open(ROOT + 'medical_segmentation_pytorch_amd/' + f).read(), f
print('patched')
