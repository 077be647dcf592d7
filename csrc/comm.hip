// Low-latency intra-node all-reduce over peer memory (xGMI) for the SyncBN statistic exchanges
// (the reference's SyncBatchNorm issues 584 tiny blocking collectives per step,
// /root/reference/utils/parallel.py:37-38).  RCCL's latency floor for a few-KB all-reduce is tens of us;
// here one kernel does the whole exchange with every rank's buffer mapped into every process (hipIpc).
//
// Every rank owns one exchange buffer in its own HBM, allocated uncached (fine-grained, MTYPE UC) and
// exported with hipIpcGetMemHandle; every other rank maps it with hipIpcOpenMemHandle.  Layout:
//   [0, 8*kCommMaxRanks)        flag[s]: the epoch rank s last delivered into THIS buffer
//   [kCommDataOff, ...)         data[parity][s][cap] fp64: rank s's contribution of the epoch
// One exchange (epoch e = local device counter + 1, identical on every rank because every rank runs the
// same sequence of exchanges):
//   1. push: the block writes its input row into slot [e&1][rank] of EVERY rank's buffer (one hop over
//      xGMI to each peer; a ring needs 2(n-1) dependent hops) with system-scope stores;
//   2. signal: release-store flag[rank] = e into every buffer;
//   3. wait: acquire-poll the local flag[s] >= e for every s (bounded: a peer that never arrives turns
//      the result into NaN and bumps an error word instead of hanging the GPU);
//   4. reduce: out = sum over s = 0..n-1 IN RANK ORDER of the local slots -> bitwise-identical results
//      on every rank (RCCL's ring order differs per rank position).
// Two parity slots make the reuse safe: a rank can only start epoch e+2 (rewriting parity e&1) after it
// saw every rank's epoch-(e+1) flag, which each rank sets only after finishing its epoch-e reduce.
// The epoch counter lives in device memory and is advanced by the kernel itself, so the exchange can be
// captured in a hipGraph and replayed (a host-side epoch would be frozen into the graph).
// No scalar-cache stores anywhere: flags and data move with per-lane (vector) system-scope atomics.
#include <cstring>

#include "common.h"
#include "launchers.h"

namespace {

constexpr int kCommBlock = 256;

DEVI void st_sys(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
DEVI unsigned long long ld_sys(const unsigned long long* p) {
  return __hip_atomic_load(const_cast<unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ``in`` and ``out`` may alias (the engine reduces in place): every load of ``in`` happens in step 1, before
// the barrier that precedes the first store to ``out`` in step 4.
// ``epoch`` = the state row: [0] epoch, and with ``nstate`` >= 4 the wait instrumentation [1] sum of the
// per-exchange spin time before the last peer's flag arrived (wall-clock ticks), [2] exchanges, [3] the max.
__global__ __launch_bounds__(kCommBlock) void oneshot_allreduce_kernel(const double* in, double* out, long n,
                                                                       CommPeers peers, int rank, int world,
                                                                       long cap, unsigned long long* epoch,
                                                                       int nstate, int* err, long long timeout) {
  __shared__ unsigned long long s_e;
  __shared__ int s_fail;
  __shared__ unsigned int s_wait;
  const int tid = threadIdx.x;
  if (tid == 0) {
    s_e = epoch[0] + 1ull;
    s_fail = 0;
    s_wait = 0u;
  }
  __syncthreads();
  const unsigned long long e = s_e;
  const long slot = (long)(e & 1ull) * world;
  // 1. push this rank's row into slot [parity][rank] of every rank's buffer
  const unsigned long long* src = reinterpret_cast<const unsigned long long*>(in);
  for (int p = 0; p < world; ++p) {
    unsigned long long* dst =
        reinterpret_cast<unsigned long long*>(peers.buf[p] + kCommDataOff) + (slot + rank) * cap;
    for (long i = tid; i < n; i += kCommBlock) st_sys(dst + i, src[i]);
  }
  __threadfence_system();
  __syncthreads();
  // 2. signal: lane p stores this rank's flag into rank p's buffer (release: orders the data above)
  if (tid < world) {
    unsigned long long* f = reinterpret_cast<unsigned long long*>(peers.buf[tid]) + rank;
    __hip_atomic_store(f, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 3. wait for every rank's flag in the local buffer (bounded spin)
  if (tid < world) {
    const unsigned long long* f = reinterpret_cast<const unsigned long long*>(peers.buf[rank]) + tid;
    const long long t0 = wall_clock64();
    long long t1 = t0;
    while (__hip_atomic_load(const_cast<unsigned long long*>(f), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      t1 = wall_clock64();
      if (t1 - t0 > timeout) {
        s_fail = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    atomicMax(&s_wait, (unsigned int)min(t1 - t0, 0x7fffffffLL));   // LDS atomic
  }
  __syncthreads();
  // 4. reduce in rank order (system-scope loads: the slots were written by other agents)
  const unsigned long long* mine = reinterpret_cast<const unsigned long long*>(peers.buf[rank] + kCommDataOff) + slot * cap;
  const bool fail = s_fail != 0;
  for (long i = tid; i < n; i += kCommBlock) {
    double acc = __longlong_as_double((long long)ld_sys(mine + i));
    for (int s = 1; s < world; ++s) acc += __longlong_as_double((long long)ld_sys(mine + (long)s * cap + i));
    out[i] = fail ? __builtin_nan("") : acc;
  }
  if (tid == 0) {
    epoch[0] = e;
    if (nstate >= 4) {   // (this kernel is the only writer of the row: plain vector read-modify-write)
      epoch[1] += s_wait;
      epoch[2] += 1ull;
      epoch[3] = max(epoch[3], (unsigned long long)s_wait);
    }
    if (fail) atomicAdd(err, 1);
  }
}

}  // namespace

long comm_buffer_bytes(long cap, int world) { return kCommDataOff + 2L * world * cap * (long)sizeof(double); }

int comm_alloc(long bytes, void** ptr, void* handle64) {
  if (hipExtMallocWithFlags(ptr, (size_t)bytes, hipDeviceMallocUncached) != hipSuccess) return 1;
  if (hipMemset(*ptr, 0, (size_t)bytes) != hipSuccess) return 2;
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, *ptr) != hipSuccess) return 4;
  static_assert(sizeof(hipIpcMemHandle_t) <= kCommHandleBytes, "IPC handle size");
  memcpy(handle64, &h, sizeof(h));
  return 0;
}

int comm_open(const void* handle64, void** ptr) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle64, sizeof(h));
  return hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess) == hipSuccess ? 0 : 1;
}

void comm_close(void* ptr) { (void)hipIpcCloseMemHandle(ptr); }
void comm_free(void* ptr) { (void)hipFree(ptr); }

void oneshot_allreduce(const double* in, double* out, long n, const CommPeers& peers, int rank, int world, long cap,
                       unsigned long long* epoch, int nstate, int* err, long long timeout, hipStream_t s) {
  hipLaunchKernelGGL(oneshot_allreduce_kernel, dim3(1), dim3(kCommBlock), 0, s, in, out, n, peers, rank, world, cap,
                     epoch, nstate, err, timeout);
}
