// One-shot all-reduce for small messages between the GPUs of one node, over peer-mapped HBM.
//
// RCCL's ring all-reduce of a ~31 KB KMeans partial-sum message (k=100 centres x 153 features + counts,
// k_means.py:83-87 every Lloyd iteration) costs 2*(world-1) dependent link hops.  Over xGMI every
// GPU maps every other GPU's memory directly (7 point-to-point links), so a small message is
// reduced in ONE kernel: each rank copies its input into its own registered buffer, tells every peer
// "block b of my data is ready" by storing the call's epoch into that peer's flag slot, waits until
// all peers have reached at least the same call for block b, then reads block b from all world buffers over the links
// and sums it locally.  One launch, one flag round trip, world-1 link reads per element.
//
// Registered buffer of each rank (hipMalloc'd once, exported with hipIpcGetMemHandle, opened by the
// peers with hipIpcOpenMemHandle):
//   [0, IPC_FLAG_BYTES)        uint32 flag[block][src rank] = epoch of the last signal
//   [IPC_FLAG_BYTES, +cap)     data slot 0
//   [.. + cap, + 2*cap)        data slot 1
// Call k writes slot k&1.  Passing call k-1's flag wait means every peer has started its call k-1
// kernel, so (one stream per rank) its call k-2 kernel — the last reader of slot k&1 — has finished:
// two slots and one flag round trip per call are enough.  Epochs strictly increase and a wait passes on
// a flag at or past its own epoch (wrap-safe compare): a peer that has already finished call k and
// signalled call k+1 overwrote the k signal with k+1, which still releases the call-k waiter, and it
// cannot get to call k+2 (the next writer of this call's slot) before this rank signals k+1.
//
// Memory ordering: data is written with plain stores, then made visible at system scope
// (__threadfence_system) before the signalling store-release; the waiting side uses system-scope
// acquire loads on its own flags and reads peer data with system-scope relaxed loads (always
// coherent over the links).  All stores are ordinary vector-memory stores.  The flag wait is bounded
// (spin_limit polls): on timeout the kernel records 1 in *err and finishes, so the grid always
// drains; the host checks *err (parallel/ipc.py).
#include "common.h"

namespace {

constexpr int IPC_MAXW = 16;
constexpr int IPC_MAXB = 64;
constexpr long IPC_FLAG_BYTES = (long)IPC_MAXB * IPC_MAXW * 4;

struct Peers {
  char* base[IPC_MAXW];
};

template <typename T>
PTG_DEV T sys_load(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <typename T>
__global__ __launch_bounds__(256) void ipc_allreduce_k(const T* in, T* out, long n,
                                                       Peers peers, int world, int rank, long cap, uint32_t epoch,
                                                       int* __restrict__ err, long long spin_limit) {
  const int b = blockIdx.x, tid = threadIdx.x;
  const long per = (n + gridDim.x - 1) / gridDim.x;
  const long lo = min(n, (long)b * per), hi = min(n, lo + per);
  const long slot_off = IPC_FLAG_BYTES + (long)(epoch & 1u) * cap;
  T* mine = (T*)(peers.base[rank] + slot_off);
  for (long i = lo + tid; i < hi; i += 256) mine[i] = in[i];
  __threadfence_system();  // this thread's slot writes reach memory before any signal
  __syncthreads();
  if (tid < world) {
    uint32_t* f = (uint32_t*)peers.base[tid] + b * IPC_MAXW + rank;
    __hip_atomic_store(f, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (tid < world) {
    const uint32_t* f = (const uint32_t*)peers.base[rank] + b * IPC_MAXW + tid;
    long long it = 0;
    // at-or-past, wrap-safe: a fast peer may already have signalled call epoch+1 into this slot
    // (it passed its call-epoch wait, so it has read nothing of ours that we are about to reuse)
    while ((int)(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      if (++it > spin_limit) {
        atomicOr(err, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  for (long i = lo + tid; i < hi; i += 256) {
    T acc = (T)0;
    for (int p = 0; p < world; ++p) acc += sys_load((const T*)(peers.base[p] + slot_off) + i);
    out[i] = acc;
  }
}

}  // namespace

extern "C" {

// layout constants for the host side (parallel/ipc.py): flag region bytes, max ranks
int ptg_ipc_flag_bytes() { return (int)IPC_FLAG_BYTES; }
int ptg_ipc_max_world() { return IPC_MAXW; }

int ptg_ipc_alloc(long bytes, void** out_ptr, void* out_handle) {
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, (size_t)bytes);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(p, 0, (size_t)bytes);
  if (e != hipSuccess) return (int)e;
  e = hipDeviceSynchronize();
  if (e != hipSuccess) return (int)e;
  e = hipIpcGetMemHandle((hipIpcMemHandle_t*)out_handle, p);
  if (e != hipSuccess) return (int)e;
  *out_ptr = p;
  return 0;
}

int ptg_ipc_open(void* handle, void** out_ptr) {
  hipIpcMemHandle_t h;
  __builtin_memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(out_ptr, h, hipIpcMemLazyEnablePeerAccess);
}

int ptg_ipc_close(void* p) { return (int)hipIpcCloseMemHandle(p); }
int ptg_ipc_free(void* p) { return (int)hipFree(p); }
int ptg_ipc_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }

// in/out: n elements (dtype 0 = fp32, 1 = fp64, 2 = int64); peer_ptrs: host array of world buffer
// base addresses (this rank's own buffer at index rank); in may equal out.
int ptg_ipc_allreduce(const void* in, void* out, long n, int dtype, const void* peer_ptrs, int world,
                                 int rank, long cap, int epoch, int* err, long spin_limit, hipStream_t stream) {
  const long esz = dtype == 0 ? 4 : 8;
  if (world < 1 || world > IPC_MAXW || rank < 0 || rank >= world || n < 0 || n * esz > cap) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  Peers peers;
  const unsigned long long* pp = (const unsigned long long*)peer_ptrs;
  for (int i = 0; i < IPC_MAXW; ++i) peers.base[i] = i < world ? (char*)pp[i] : nullptr;
  for (int i = 0; i < world; ++i)
    if (!peers.base[i]) return (int)hipErrorInvalidValue;
  const int nb = (int)min((long)IPC_MAXB, max(1L, (n + 2047) / 2048));
  const uint32_t ep = (uint32_t)epoch;
  if (dtype == 0)
    hipLaunchKernelGGL(ipc_allreduce_k<float>, dim3(nb), dim3(256), 0, stream, (const float*)in, (float*)out, n, peers,
                       world, rank, cap, ep, err, (long long)spin_limit);
  else if (dtype == 1)
    hipLaunchKernelGGL(ipc_allreduce_k<double>, dim3(nb), dim3(256), 0, stream, (const double*)in, (double*)out, n,
                       peers, world, rank, cap, ep, err, (long long)spin_limit);
  else
    hipLaunchKernelGGL(ipc_allreduce_k<long long>, dim3(nb), dim3(256), 0, stream, (const long long*)in,
                       (long long*)out, n, peers, world, rank, cap, ep, err, (long long)spin_limit);
  PTG_RETURN_LAUNCH();
}

}  // extern "C"
