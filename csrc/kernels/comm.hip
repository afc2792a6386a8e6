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

// ---- collective stand-ins of the simulated-world mode (distribute/strategy.py, PTG_SIM_WORLD=N):
// one rank runs rank 0's kernel sequence of an N-rank sharded update with its collectives replaced
// by local kernels that move the same local HBM bytes.  Reduce-scatter: read every chunk of the
// bucket (a ring sends N-1 of them), write the owned shard = own_scale * chunk 0 (+ w_peer * the other
// chunks, 0 for "N ranks with identical data": their chunk-0 partials equal ours).
__global__ __launch_bounds__(256) void sim_rs_k(const float4* __restrict__ g, float4* __restrict__ out, long cnt4,
                                                int nchunks, float own_scale, float w_peer) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < cnt4; i += (long)gridDim.x * 256) {
    float4 a = g[i], p = float4{0.f, 0.f, 0.f, 0.f};
    for (int r = 1; r < nchunks; ++r) {
      const float4 b = g[(long)r * cnt4 + i];
      p.x += b.x; p.y += b.y; p.z += b.z; p.w += b.w;
    }
    out[i] = float4{own_scale * a.x + w_peer * p.x, own_scale * a.y + w_peer * p.y, own_scale * a.z + w_peer * p.z,
                    own_scale * a.w + w_peer * p.w};
  }
}

// All-gather: the N-1 peer chunks of a bucket land in local HBM; here they are rewritten in place
// (read + write of (N-1)/N of the bucket: the received bytes, plus a read the real gather does not do)
__global__ __launch_bounds__(256) void sim_ag_k(uint4* __restrict__ buf, long lo4, long hi4, uint32_t mask) {
  for (long i = lo4 + blockIdx.x * 256L + threadIdx.x; i < hi4; i += (long)gridDim.x * 256) {
    uint4 v = buf[i];
    v.x ^= mask; v.y ^= mask; v.z ^= mask; v.w ^= mask;
    buf[i] = v;
  }
}

// ---- parameter-server piece copies (distribute/strategy.py _PSPlan): a model's variables are cut
// into pieces placed on PS owners; push / pull move every piece between the flat parameter store and
// the owners' packed segments.  ONE launch moves all pieces of a step (the pieces are pre-split into
// chunks of <= 64K elements on the host, one workgroup per chunk), converting fp32 <-> bf16 on the
// way; a base may be a peer's IPC-mapped window (reads / writes over xGMI).
struct PieceBases {
  char* base[IPC_MAXW];
};

// sys: the source is memory another agent writes (a peer's window, or this rank's window written by
// peers): element loads are system-scope, so no line a cache kept from an earlier read is returned
// (hipMalloc memory is coarse-grained; only the scope of the access makes a peer's write visible)
template <typename T>
PTG_DEV T ld_sys(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// table: 5 longs per chunk = src base index, src element offset, dst base index, dst element offset, n
template <bool SYS>
__global__ __launch_bounds__(256) void piece_copy_k(PieceBases src, int src_bf, PieceBases dst, int dst_bf,
                                                    const long* __restrict__ table, int nchunks) {
  for (int c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const long* e = table + 5L * c;
    const char* sb = src.base[e[0]];
    char* db = dst.base[e[2]];
    const long so = e[1], dof = e[3], n = e[4];
    if (src_bf == dst_bf && !src_bf) {
      const uint32_t* sp = (const uint32_t*)sb + so;
      for (long i = threadIdx.x; i < n; i += 256) ((uint32_t*)db)[dof + i] = SYS ? ld_sys(sp + i) : sp[i];
    } else if (src_bf == dst_bf) {
      const uint16_t* sp = (const uint16_t*)sb + so;
      for (long i = threadIdx.x; i < n; i += 256) ((uint16_t*)db)[dof + i] = SYS ? ld_sys(sp + i) : sp[i];
    } else if (src_bf) {  // bf16 -> fp32
      const uint16_t* sp = (const uint16_t*)sb + so;
      for (long i = threadIdx.x; i < n; i += 256) {
        const uint16_t u = SYS ? ld_sys(sp + i) : sp[i];
        ((float*)db)[dof + i] = __uint_as_float((uint32_t)u << 16);
      }
    } else {  // fp32 -> bf16
      const uint32_t* sp = (const uint32_t*)sb + so;
      for (long i = threadIdx.x; i < n; i += 256) {
        const uint32_t u = SYS ? ld_sys(sp + i) : sp[i];
        ((uint16_t*)db)[dof + i] = (uint16_t)f2bf(__uint_as_float(u));
      }
    }
  }
}

}  // namespace

extern "C" {

// srcs / dsts: host arrays of up to 16 base addresses; table: device array of 5 * nchunks longs
int ptg_piece_copy(const void* srcs, int nsrc, int src_bf16, const void* dsts, int ndst, int dst_bf16,
                   const long* table, int nchunks, int sys, hipStream_t stream) {
  if (nsrc < 1 || nsrc > IPC_MAXW || ndst < 1 || ndst > IPC_MAXW || nchunks < 0) return (int)hipErrorInvalidValue;
  if (nchunks == 0) return 0;
  PieceBases sb, db;
  const unsigned long long* sp = (const unsigned long long*)srcs;
  const unsigned long long* dp = (const unsigned long long*)dsts;
  for (int i = 0; i < IPC_MAXW; ++i) {
    sb.base[i] = i < nsrc ? (char*)sp[i] : nullptr;
    db.base[i] = i < ndst ? (char*)dp[i] : nullptr;
  }
  const int grid = nchunks < 4096 ? nchunks : 4096;
  if (sys)
    hipLaunchKernelGGL(piece_copy_k<true>, dim3(grid), dim3(256), 0, stream, sb, src_bf16, db, dst_bf16, table, nchunks);
  else
    hipLaunchKernelGGL(piece_copy_k<false>, dim3(grid), dim3(256), 0, stream, sb, src_bf16, db, dst_bf16, table, nchunks);
  PTG_RETURN_LAUNCH();
}

// export a pointer inside a device allocation (e.g. a torch tensor): IPC handle of its allocation +
// the byte offset of the pointer in it (peers open the handle and add the offset)
int ptg_ipc_export(void* ptr, void* out_handle, long* out_offset) {
  void* base = nullptr;
  size_t size = 0;
  hipError_t e = hipMemGetAddressRange(&base, &size, ptr);
  if (e != hipSuccess) return (int)e;
  e = hipIpcGetMemHandle((hipIpcMemHandle_t*)out_handle, base);
  if (e != hipSuccess) return (int)e;
  *out_offset = (long)((char*)ptr - (char*)base);
  return 0;
}

int ptg_sim_reduce_scatter(const float* g, float* out, long cnt, int nchunks, float own_scale, float w_peer,
                           hipStream_t stream) {
  if (cnt % 4 || nchunks < 1) return (int)hipErrorInvalidValue;
  const long cnt4 = cnt / 4;
  if (cnt4 == 0) return 0;
  const int grid = (int)min(2048L, (cnt4 + 255) / 256);
  hipLaunchKernelGGL(sim_rs_k, dim3(grid), dim3(256), 0, stream, (const float4*)g, (float4*)out, cnt4, nchunks,
                     own_scale, w_peer);
  PTG_RETURN_LAUNCH();
}

// buf: the bucket's first byte; bytes [lo, hi) (16-B multiples) are the peer chunks
int ptg_sim_all_gather(void* buf, long lo, long hi, hipStream_t stream) {
  if (lo % 16 || hi % 16 || hi < lo) return (int)hipErrorInvalidValue;
  const long lo4 = lo / 16, hi4 = hi / 16;
  if (hi4 == lo4) return 0;
  const int grid = (int)min(2048L, (hi4 - lo4 + 255) / 256);
  hipLaunchKernelGGL(sim_ag_k, dim3(grid), dim3(256), 0, stream, (uint4*)buf, lo4, hi4, 0u);
  PTG_RETURN_LAUNCH();
}

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

int ptg_stream_destroy(void* st) { return (int)hipStreamDestroy((hipStream_t)st); }

// Cross-stream fork / join events of the training step's side stream (nn/streams.py).  A default HIP
// event record ends with a SYSTEM-scope release (cache writeback + invalidate, so the host could read
// device memory): on the step's stream that stalled the next kernel ~6.5 us per fork
// (profiles/r5_cnn_b1_b256_gantt.txt gaps).  The two streams share one device, so a device-scope
// release is all the ordering needs (hipEventDisableSystemFence).
int ptg_event_create_device(void** out) {
  hipEvent_t e;
  const hipError_t rc = hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence);
  *out = rc == hipSuccess ? (void*)e : nullptr;
  return (int)rc;
}
int ptg_event_destroy(void* e) { return (int)hipEventDestroy((hipEvent_t)e); }
int ptg_event_record(void* e, hipStream_t s) { return (int)hipEventRecord((hipEvent_t)e, s); }
int ptg_stream_wait_event(void* e, hipStream_t s) { return (int)hipStreamWaitEvent(s, (hipEvent_t)e, 0); }

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
