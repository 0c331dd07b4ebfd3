#include "shm_ring.h"

#include <linux/futex.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>
#include <chrono>
#include <cstring>
#include <thread>

namespace mb {

static long futex(std::atomic<uint32_t>* addr, int op, uint32_t val, const timespec* ts) {
  return syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), op, val, ts, nullptr, 0);
}

IndexRing::IndexRing(void* mem, size_t capacity, bool init) {
  hdr_ = reinterpret_cast<RingHeader*>(mem);
  cells_ = reinterpret_cast<RingCell*>(reinterpret_cast<char*>(mem) + sizeof(RingHeader));
  if (init) {
    hdr_->head.store(0);
    hdr_->tail.store(0);
    hdr_->futex.store(0);
    hdr_->closed.store(0);
    hdr_->capacity = capacity;
    for (size_t i = 0; i < capacity; ++i) {
      cells_[i].seq.store(i);
      cells_[i].value = -1;
    }
    std::atomic_thread_fence(std::memory_order_seq_cst);
  }
}

bool IndexRing::try_push(int64_t v) {
  const uint64_t cap = hdr_->capacity;
  uint64_t pos = hdr_->tail.load(std::memory_order_relaxed);
  for (;;) {
    RingCell& c = cells_[pos % cap];
    uint64_t seq = c.seq.load(std::memory_order_acquire);
    int64_t dif = (int64_t)seq - (int64_t)pos;
    if (dif == 0) {
      if (hdr_->tail.compare_exchange_weak(pos, pos + 1, std::memory_order_relaxed)) {
        c.value = v;
        c.seq.store(pos + 1, std::memory_order_release);
        wake();
        return true;
      }
    } else if (dif < 0) {
      return false;  // full
    } else {
      pos = hdr_->tail.load(std::memory_order_relaxed);
    }
  }
}

bool IndexRing::try_pop(int64_t* v) {
  const uint64_t cap = hdr_->capacity;
  uint64_t pos = hdr_->head.load(std::memory_order_relaxed);
  for (;;) {
    RingCell& c = cells_[pos % cap];
    uint64_t seq = c.seq.load(std::memory_order_acquire);
    int64_t dif = (int64_t)seq - (int64_t)(pos + 1);
    if (dif == 0) {
      if (hdr_->head.compare_exchange_weak(pos, pos + 1, std::memory_order_relaxed)) {
        *v = c.value;
        c.seq.store(pos + cap, std::memory_order_release);
        wake();
        return true;
      }
    } else if (dif < 0) {
      return false;  // empty
    } else {
      pos = hdr_->head.load(std::memory_order_relaxed);
    }
  }
}

void IndexRing::wake() {
  hdr_->futex.fetch_add(1, std::memory_order_release);
  futex(&hdr_->futex, FUTEX_WAKE, 0x7fffffff, nullptr);
}

bool IndexRing::wait(uint32_t seen, double timeout_s) {
  timespec ts, *tsp = nullptr;
  // wake up at least every 50 ms so 'closed' and deadlines are re-checked
  double slice = timeout_s < 0 ? 0.05 : (timeout_s < 0.05 ? timeout_s : 0.05);
  ts.tv_sec = (time_t)slice;
  ts.tv_nsec = (long)((slice - (double)ts.tv_sec) * 1e9);
  tsp = &ts;
  futex(&hdr_->futex, FUTEX_WAIT, seen, tsp);
  return true;
}

bool IndexRing::push(int64_t v, double timeout_s) {
  auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    uint32_t seen = hdr_->futex.load(std::memory_order_acquire);
    if (try_push(v)) return true;
    if (closed()) return false;
    double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (timeout_s >= 0 && el >= timeout_s) return false;
    wait(seen, timeout_s < 0 ? -1.0 : timeout_s - el);
  }
}

bool IndexRing::pop(int64_t* v, double timeout_s) {
  auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    uint32_t seen = hdr_->futex.load(std::memory_order_acquire);
    if (try_pop(v)) return true;
    if (closed()) return false;
    double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (timeout_s >= 0 && el >= timeout_s) return false;
    wait(seen, timeout_s < 0 ? -1.0 : timeout_s - el);
  }
}

size_t IndexRing::size() const {
  uint64_t t = hdr_->tail.load(), h = hdr_->head.load();
  return t > h ? (size_t)(t - h) : 0;
}

void IndexRing::close() {
  hdr_->closed.store(1);
  wake();
}

uint64_t seqlock_write_begin(std::atomic<uint64_t>* ver) {
  uint64_t v = ver->load(std::memory_order_relaxed) + 1;  // odd
  ver->store(v, std::memory_order_relaxed);
  std::atomic_thread_fence(std::memory_order_release);
  return v;
}

void seqlock_write_end(std::atomic<uint64_t>* ver) {
  std::atomic_thread_fence(std::memory_order_release);
  ver->store(ver->load(std::memory_order_relaxed) + 1, std::memory_order_release);
}

// The protected region is copied through relaxed atomic 8-byte accesses on both sides
// (plain moves on x86), so concurrent readers and the writer never race in the C++
// memory-model sense; the version check makes a torn copy detectable. n % 8 tail bytes
// go through atomic byte accesses.
static void atomic_copy_out(const void* src, void* dst, size_t n) {
  const uint64_t* s = (const uint64_t*)src;
  uint64_t* d = (uint64_t*)dst;
  const size_t w = n / 8;
  for (size_t i = 0; i < w; ++i) d[i] = __atomic_load_n(s + i, __ATOMIC_RELAXED);
  for (size_t i = w * 8; i < n; ++i)
    ((uint8_t*)dst)[i] = __atomic_load_n((const uint8_t*)src + i, __ATOMIC_RELAXED);
}
static void atomic_copy_in(const void* src, void* dst, size_t n) {
  const uint64_t* s = (const uint64_t*)src;
  uint64_t* d = (uint64_t*)dst;
  const size_t w = n / 8;
  for (size_t i = 0; i < w; ++i) __atomic_store_n(d + i, s[i], __ATOMIC_RELAXED);
  for (size_t i = w * 8; i < n; ++i)
    __atomic_store_n((uint8_t*)dst + i, ((const uint8_t*)src)[i], __ATOMIC_RELAXED);
}

void seqlock_write(std::atomic<uint64_t>* ver, const void* src, void* dst, size_t n) {
  seqlock_write_begin(ver);
  atomic_copy_in(src, dst, n);
  seqlock_write_end(ver);
}

uint64_t seqlock_read(const std::atomic<uint64_t>* ver, const void* src, void* dst, size_t n,
                      int max_tries) {
  for (int i = 0; i < max_tries; ++i) {
    uint64_t v0 = ver->load(std::memory_order_acquire);
    if (v0 & 1) { std::this_thread::yield(); continue; }
    atomic_copy_out(src, dst, n);
    std::atomic_thread_fence(std::memory_order_acquire);
    uint64_t v1 = ver->load(std::memory_order_relaxed);
    if (v0 == v1) return v0 + 1;  // version + 1, so 0 always means failure
  }
  return 0;
}

}  // namespace mb
