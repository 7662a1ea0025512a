// shm_exchange.cpp — the elastic service's per-step control exchange over node-local shared
// memory (libdml_host.so; parallel/elastic.py ElasticGroup.exchange).
//
// Every rank of an epoch contributes one fixed-size record per step and receives all of
// them (all-gather semantics). The service runs one rank per GPU of ONE node, so the
// exchange is a shared-memory handshake instead of a gloo gather + broadcast: rank r copies
// its record into slot[step & 1][r] and publishes `step` in its own cache line (release);
// it then waits (acquire) until every rank's published step reaches `step` and copies the
// slots out. Two slot banks suffice: a rank can only write bank (s & 1) again at step s + 2,
// after every rank has published s + 1, i.e. finished reading step s.
//
// The wait runs in native code with the GIL released (ctypes), so a busy Python thread of
// the same process (the store's asyncio loop, the output writer) no longer stretches every
// collective by several GIL switch intervals (measured with gloo: 0.1 ms idle, 40 ms per
// world-1 exchange next to a spinning Python thread). A wait returns 1 after timeout_us so
// the caller can consult the failure detector (a dead rank never publishes) and call again;
// a repeated call for the same step does not publish twice.
//
// Reference: the leader's UDP round trips per task / ACK (worker.py:297, 531, 989-1026).
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <cstdint>
#include <cstring>
#include <string>

namespace {

constexpr uint64_t kMagic = 0x444d4c5348584348ull;  // "DMLSHXCH"
constexpr int kLine = 64;

struct Header {
  uint64_t magic;
  int32_t world;
  int32_t rec_cap;
};

struct Handle {
  char* base = nullptr;
  size_t bytes = 0;
  int world = 0;
  int rec_cap = 0;
  std::string name;
  uint64_t* seq(int r) const { return (uint64_t*)(base + kLine * (1 + r)); }
  char* slot(int bank, int r) const {
    return base + kLine * (1 + world) + ((size_t)bank * world + r) * (size_t)rec_cap;
  }
};

inline double now_us() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

}  // namespace

extern "C" {

// Open (creating if needed) the exchange segment `name` (a POSIX shm name, "/..."), sized
// for `world` ranks and records of up to rec_cap bytes. Every rank of the epoch calls it;
// the creator's zero-filled sequence numbers start every rank at step 0.
void* dml_shm_open(const char* name, int world, int rec_cap) {
  if (world < 1 || world > 1024 || rec_cap < 8 || rec_cap % kLine) return nullptr;
  const size_t bytes = (size_t)kLine * (1 + world) + (size_t)2 * world * rec_cap;
  bool creator = true;
  int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0) {
    creator = false;
    fd = shm_open(name, O_RDWR, 0600);
  }
  if (fd < 0) return nullptr;
  if (creator) {
    if (ftruncate(fd, (off_t)bytes) != 0) {
      close(fd);
      return nullptr;
    }
  } else {  // the creator may not have sized it yet: never map (and touch) a short file
    struct stat st;
    const double t0 = now_us();
    while (fstat(fd, &st) == 0 && (size_t)st.st_size < bytes && now_us() - t0 < 10e6) {
      timespec ts{0, 100000};
      nanosleep(&ts, nullptr);
    }
    if (fstat(fd, &st) != 0 || (size_t)st.st_size < bytes) {
      close(fd);
      return nullptr;
    }
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return nullptr;
  Header* hd = (Header*)p;
  if (creator) {
    hd->world = world;
    hd->rec_cap = rec_cap;
    __atomic_store_n(&hd->magic, kMagic, __ATOMIC_RELEASE);
  } else {
    const double t0 = now_us();
    while (__atomic_load_n(&hd->magic, __ATOMIC_ACQUIRE) != kMagic && now_us() - t0 < 10e6) sched_yield();
  }
  if (__atomic_load_n(&hd->magic, __ATOMIC_ACQUIRE) != kMagic || hd->world != world || hd->rec_cap != rec_cap) {
    munmap(p, bytes);  // another geometry (or a creator that died half-way): refuse
    return nullptr;
  }
  Handle* h = new Handle();
  h->base = (char*)p;
  h->bytes = bytes;
  h->world = world;
  h->rec_cap = rec_cap;
  h->name = name;
  return h;
}

// Publish `rec` (rec_bytes) as rank `rank`'s record of `step` (>= 1, one more than the
// previous exchange of this segment) and gather every rank's record of that step into
// out[world][rec_bytes]. 0: done; 1: timed out waiting (call again with the same step);
// -1: bad arguments.
int dml_shm_exchange(void* hp, int rank, long long step, const void* rec, int rec_bytes, void* out,
                     int timeout_us) {
  Handle* h = (Handle*)hp;
  if (!h || rank < 0 || rank >= h->world || rec_bytes > h->rec_cap || step < 1) return -1;
  const int bank = (int)(step & 1);
  uint64_t* mine = h->seq(rank);
  if (__atomic_load_n(mine, __ATOMIC_ACQUIRE) < (uint64_t)step) {  // not yet published (a retry skips this)
    std::memcpy(h->slot(bank, rank), rec, (size_t)rec_bytes);
    __atomic_store_n(mine, (uint64_t)step, __ATOMIC_RELEASE);
  }
  const double t0 = now_us();
  for (int r = 0; r < h->world; ++r) {
    int spins = 0;
    while (__atomic_load_n(h->seq(r), __ATOMIC_ACQUIRE) < (uint64_t)step) {
      if (++spins < 64) {
        __builtin_ia32_pause();
      } else if (spins < 256) {
        sched_yield();
      } else {
        timespec ts{0, 5000};  // 5 us: the waiting rank leaves its core to the others
        nanosleep(&ts, nullptr);
      }
      if ((spins & 15) == 0 && now_us() - t0 > timeout_us) return 1;
    }
  }
  for (int r = 0; r < h->world; ++r)
    std::memcpy((char*)out + (size_t)r * rec_bytes, h->slot(bank, r), (size_t)rec_bytes);
  return 0;
}

void dml_shm_close(void* hp, int unlink_name) {
  Handle* h = (Handle*)hp;
  if (!h) return;
  munmap(h->base, h->bytes);
  if (unlink_name) shm_unlink(h->name.c_str());
  delete h;
}

int dml_shm_unlink(const char* name) { return shm_unlink(name); }

}  // extern "C"
