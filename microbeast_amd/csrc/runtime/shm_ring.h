// Cross-process bounded MPMC index ring + seqlock, living in caller-provided
// shared memory (POSIX shm mapped by Python).
//
// Replaces the reference's spawn-context multiprocessing.Queue pair
// (free_queue / full_queue, reference microbeast.py:169-175, 59-65, 105;
// libs/utils.py:183-192, 211-213) which pickled one int per message through a
// pipe and was busy-polled with empty()/qsize(). Here: Vyukov per-cell
// sequence numbers (lock-free), futex sleep when empty/full, bounded waits.
//
// The seqlock replaces the torn-read-prone in-place load_state_dict into a
// shared nn.Module (reference libs/utils.py:337) for CPU actors.
#pragma once
#include <atomic>
#include <cstddef>
#include <cstdint>

namespace mb {

struct RingCell {
  std::atomic<uint64_t> seq;
  int64_t value;
};

struct RingHeader {
  std::atomic<uint64_t> head;    // next pop
  std::atomic<uint64_t> tail;    // next push
  std::atomic<uint32_t> futex;   // bumped on every push/pop
  std::atomic<uint32_t> closed;
  uint64_t capacity;
  uint64_t pad[3];
};

class IndexRing {
 public:
  static size_t bytes_needed(size_t capacity) {
    return sizeof(RingHeader) + capacity * sizeof(RingCell);
  }
  // init=true: the creating process formats the memory.
  IndexRing(void* mem, size_t capacity, bool init);
  bool try_push(int64_t v);
  bool try_pop(int64_t* v);
  // timeout_s < 0: wait forever. Returns false on timeout or when closed.
  bool push(int64_t v, double timeout_s);
  bool pop(int64_t* v, double timeout_s);
  size_t size() const;
  size_t capacity() const { return hdr_->capacity; }
  void close();
  bool closed() const { return hdr_->closed.load() != 0; }

 private:
  RingHeader* hdr_;
  RingCell* cells_;
  void wake();
  bool wait(uint32_t seen, double timeout_s);
};

// Seqlock over a shared byte region. Writer: begin (odd) -> copy -> end (even).
uint64_t seqlock_write_begin(std::atomic<uint64_t>* ver);
void seqlock_write_end(std::atomic<uint64_t>* ver);
// begin + copy src -> dst (the shared region) + end, race-free against seqlock_read
void seqlock_write(std::atomic<uint64_t>* ver, const void* src, void* dst, size_t n);
// Copies src->dst consistently; returns (version read + 1), or 0 if it could
// not get a stable copy within max_tries.
uint64_t seqlock_read(const std::atomic<uint64_t>* ver, const void* src, void* dst, size_t n,
                      int max_tries);

}  // namespace mb
