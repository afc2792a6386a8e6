// Cross-process signalling in host shared memory for the asynchronous parameter server
// (pyspark_tf_gke_amd/distribute/ps.py _Mailbox).
//
// TF's PS runtime answers a worker's apply_gradients over gRPC (train_tf_ps.py:612-645: every
// closure's update is a round trip to the PS tasks).  Here the workers and the parameter owners of
// one node share a /dev/shm control block: a push takes a ticket with one atomic fetch-add,
// publishes (sequence, gradient scale, optimizer index) in a slot, and waits for the owner's
// applied-counter; the owner thread sleeps on the slot's sequence word.  Waiters spin briefly, then
// block in a shared (non-private) futex, so a wake-up costs one syscall instead of a TCP
// round trip to the rendezvous store.  ctypes releases the GIL around these calls.
#include <climits>
#include <cstdint>
#include <ctime>
#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>

namespace {

inline int futex_wait(int* p, int expected, long timeout_us) {
  timespec ts;
  ts.tv_sec = timeout_us / 1000000;
  ts.tv_nsec = (timeout_us % 1000000) * 1000;
  return (int)syscall(SYS_futex, p, FUTEX_WAIT, expected, &ts, nullptr, 0);
}

inline void futex_wake(int* p) { syscall(SYS_futex, p, FUTEX_WAKE, INT_MAX, nullptr, nullptr, 0); }

inline long now_us() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1000000L + ts.tv_nsec / 1000;
}

// 0 once *p >= v, 1 after timeout_us
int wait_ge(int* p, int v, long timeout_us) {
  for (int i = 0; i < 2000; ++i) {
    if (__atomic_load_n(p, __ATOMIC_ACQUIRE) >= v) return 0;
    __builtin_ia32_pause();
  }
  const long end = now_us() + timeout_us;
  for (;;) {
    const int cur = __atomic_load_n(p, __ATOMIC_ACQUIRE);
    if (cur >= v) return 0;
    const long left = end - now_us();
    if (left <= 0) return 1;
    futex_wait(p, cur, left < 50000 ? left : 50000);
  }
}

struct Slot {  // one 64-byte line of the control block
  int seq;     // ticket + 1 once published
  int oi;      // optimizer index (-1: the model's compiled optimizer)
  double gscale;
};

}  // namespace

extern "C" {

// *old = atomic fetch-add of v to the int at p
int ptgh_shm_add(void* p, int v, int* old) {
  *old = __atomic_fetch_add((int*)p, v, __ATOMIC_ACQ_REL);
  return 0;
}

int ptgh_shm_load(void* p, int* out) {
  *out = __atomic_load_n((int*)p, __ATOMIC_ACQUIRE);
  return 0;
}

// release-store v and wake every waiter on p
int ptgh_shm_store(void* p, int v) {
  __atomic_store_n((int*)p, v, __ATOMIC_RELEASE);
  futex_wake((int*)p);
  return 0;
}

int ptgh_shm_wake(void* p) {
  futex_wake((int*)p);
  return 0;
}

// 0 once the int at p is >= v, 1 on timeout
int ptgh_shm_wait_ge(void* p, int v, long timeout_us) { return wait_ge((int*)p, v, timeout_us); }

// the payload first, then the sequence word (release) and a wake-up
int ptgh_mbox_publish(void* slot, int seq, double gscale, int oi) {
  Slot* s = (Slot*)slot;
  s->gscale = gscale;
  s->oi = oi;
  __atomic_store_n(&s->seq, seq, __ATOMIC_RELEASE);
  futex_wake(&s->seq);
  return 0;
}

// waits until the slot holds sequence >= seq: 0 and the payload, or 1 on timeout
int ptgh_mbox_take(void* slot, int seq, long timeout_us, double* gscale, int* oi) {
  Slot* s = (Slot*)slot;
  if (wait_ge(&s->seq, seq, timeout_us)) return 1;
  *gscale = s->gscale;
  *oi = s->oi;
  return 0;
}

}  // extern "C"
