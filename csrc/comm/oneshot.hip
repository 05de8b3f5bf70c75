// One-shot IPC all-reduce for SMALL gradient buckets on one node (the optional
// small-bucket path beside RCCL): every rank stages its bucket in its own IPC-exported buffer,
// publishes a sequence number into every peer's flag slot, waits until every peer's number
// has arrived in its own flags, then reads all `world` staging buffers over xGMI and sums
// them in RANK ORDER (fp32 accumulation) — the same bits on every rank, in ONE kernel.  A
// ring all-reduce pays 2(n-1) dependent steps of link latency; for a bucket of a few hundred
// KB that latency, not the ~150 GB/s per link, is the cost.  xGMI is point-to-point, so the
// n-1 peer reads of a rank run on n-1 different links at once.
//
// Protocol (seq = this rank's call count + 1, identical on every rank because every rank
// issues the same calls in the same order):
//   1. every block copies its share of src into staging half (seq & 1) — two halves, so a
//      rank never overwrites data a slow peer may still be reading: a peer reading call
//      seq's half has not yet published seq + 1, so this rank cannot start call seq + 2;
//   2. each block fences (system scope) and arrives on a local counter; the last arrival
//      writes seq into slot [rank] of every rank's flag array (remote stores, system scope);
//   3. every block waits (one lane per peer, acquire loads, s_sleep) until all `world` slots
//      of its own flag array reach seq — with a wall-clock limit (s_memrealtime, 100 MHz):
//      a missing peer sets the error word and the kernel finishes instead of hanging;
//   4. every block sums its share over the world staging halves in rank order into dst — a
//      block that timed out in 3 writes NaN over its share instead: a peer's staging half
//      may be stale, and a NaN gradient is what the optimizer's device gate skips (under DP
//      it checks the whole all-reduced gradient), so a timed-out call never applies a sum
//      of stale buffers (the error word also makes the watchdog abort the run);
//   5. the last block to finish resets the counters and stores seq (graph-replayable: no
//      host-side arguments change between calls).
// Staging buffers and flags are allocated uncached (hipDeviceMallocUncached): remote writes
// and reads then see memory, not a stale L2 line.  dtype 0 = fp32, 1 = bf16 (summed in fp32).
// Co-residency: a block past step 2 waits for the LAST block's arrival, so the call completes
// only once every one of its `blocks` workgroups has been scheduled.  Launched beside the
// step's compute kernels (which fill every CU) the late blocks start as those kernels' own
// workgroups retire — a delay, never a deadlock (no compute kernel waits on this one) — so
// keep `blocks` small (the default 16 fits in the CU slots the backward leaves free) and the
// timeout far above a step.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dgipc {

constexpr int MAXW = 8;

struct OneShotArgs {
  const void* src;
  void* dst;
  long long nvec;            // 16-byte vectors (host pads the bucket to a multiple of 16 B)
  int dtype;                 // 0 fp32, 1 bf16
  int rank, world;
  char* bufs[MAXW];          // staging (2 halves of half_bytes) of every rank (peers: IPC)
  unsigned* flags[MAXW];     // flag array [MAXW] of every rank (peers: IPC)
  long long half_bytes;
  unsigned* state;           // local: [0] calls done (seq), [1] arrive, [2] done, [3] error
  long long timeout_ticks;   // s_memrealtime ticks (100 MHz)
};

__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xFFFF0000u); }
__device__ __forceinline__ uint32_t bf_pack(float lo, float hi) {
  const uint32_t a = __builtin_bit_cast(uint16_t, (__bf16)lo);
  const uint32_t b = __builtin_bit_cast(uint16_t, (__bf16)hi);
  return a | (b << 16);
}

__global__ void __launch_bounds__(256) oneshot_allreduce_kernel(OneShotArgs a) {
  __shared__ unsigned s_seq;
  __shared__ unsigned s_last;
  const int tid = threadIdx.x;
  if (tid == 0) s_seq = __hip_atomic_load(a.state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  __syncthreads();
  const unsigned seq = s_seq;
  const long long off = (long long)(seq & 1u) * a.half_bytes;
  const long long gid = (long long)blockIdx.x * blockDim.x + tid;
  const long long stride = (long long)gridDim.x * blockDim.x;

  // 1. stage
  uint4* mine = (uint4*)(a.bufs[a.rank] + off);
  for (long long i = gid; i < a.nvec; i += stride) mine[i] = ((const uint4*)a.src)[i];
  // 2. publish
  __threadfence_system();
  __syncthreads();
  if (tid == 0) {
    const unsigned old = __hip_atomic_fetch_add(a.state + 1, 1u, __ATOMIC_ACQ_REL,
                                                __HIP_MEMORY_SCOPE_AGENT);
    s_last = old == gridDim.x - 1 ? 1u : 0u;
  }
  __syncthreads();
  if (s_last && tid < a.world)
    __hip_atomic_store(a.flags[tid] + a.rank, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  // 3. wait for every peer's data (bounded)
  __shared__ unsigned s_timeout;
  if (tid == 0) s_timeout = 0u;
  __syncthreads();
  if (tid < a.world) {
    const unsigned* f = a.flags[a.rank] + tid;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < seq) {
      __builtin_amdgcn_s_sleep(2);
      if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > a.timeout_ticks) {
        __hip_atomic_fetch_or(a.state + 3, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_timeout = 1u;   // (benign same-value race between the waiting lanes)
        break;
      }
    }
  }
  __syncthreads();
  // 4. sum in rank order (a timed-out block: NaN over its share, never a stale sum).  The NaN
  // only reaches THIS rank: a late peer that still finds this rank's flag sums normally and
  // applies its step, so the replicas can differ for the step in flight.  What keeps them
  // consistent is the error word (state[3]): the host's async-error poll (NativeComm.async_error
  // reads dp.IpcOneShot.error; the step watchdog polls it) aborts the whole job on any rank's timeout
  // before further steps are issued — the NaN only keeps this rank from applying a stale sum.
  const bool timed_out = s_timeout != 0u;
  for (long long i = gid; i < a.nvec; i += stride) {
    if (timed_out) {
      ((uint4*)a.dst)[i] = a.dtype == 0 ? uint4{0x7FC00000u, 0x7FC00000u, 0x7FC00000u, 0x7FC00000u}
                                        : uint4{0x7FC07FC0u, 0x7FC07FC0u, 0x7FC07FC0u, 0x7FC07FC0u};
      continue;
    }
    if (a.dtype == 0) {
      float4 s = {0.f, 0.f, 0.f, 0.f};
      for (int j = 0; j < a.world; ++j) {
        const float4 v = ((const float4*)(a.bufs[j] + off))[i];
        s.x += v.x;
        s.y += v.y;
        s.z += v.z;
        s.w += v.w;
      }
      ((float4*)a.dst)[i] = s;
    } else {
      float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int j = 0; j < a.world; ++j) {
        const uint4 v = ((const uint4*)(a.bufs[j] + off))[i];
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s[2 * e] += bf_lo(w[e]);
          s[2 * e + 1] += bf_hi(w[e]);
        }
      }
      ((uint4*)a.dst)[i] = uint4{bf_pack(s[0], s[1]), bf_pack(s[2], s[3]), bf_pack(s[4], s[5]),
                                 bf_pack(s[6], s[7])};
    }
  }
  // 5. the last block resets the counters and records the call
  __syncthreads();
  if (tid == 0) {
    const unsigned old = __hip_atomic_fetch_add(a.state + 2, 1u, __ATOMIC_ACQ_REL,
                                                __HIP_MEMORY_SCOPE_AGENT);
    if (old == gridDim.x - 1) {
      __hip_atomic_store(a.state + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.state + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.state, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace dgipc

// C ABI for comm.cpp (host side).  grid: blocks (constant per communicator is not required:
// the counters reset every call).
extern "C" hipError_t dg_oneshot_allreduce(const dgipc::OneShotArgs* a, int blocks,
                                           hipStream_t stream) {
  if (!a || a->world < 1 || a->world > dgipc::MAXW || a->rank < 0 || a->rank >= a->world ||
      a->nvec < 0 || a->nvec * 16 > a->half_bytes || blocks < 1 || blocks > 1024)
    return hipErrorInvalidValue;
  for (int j = 0; j < a->world; ++j)
    if (!a->bufs[j] || !a->flags[j]) return hipErrorInvalidValue;
  hipLaunchKernelGGL(dgipc::oneshot_allreduce_kernel, dim3(blocks), dim3(256), 0, stream, *a);
  return hipGetLastError();
}
