// store_io.cpp — batched file operations of the replicated store's same-node fast path
// (libdml_host.so; store/service.py spool + replica links).
//
// Every Python-level file syscall releases the GIL and must win it back before the next one:
// with a rank's serve loop, output writer and control loop all runnable, each re-acquisition
// waited out a share of the switch interval (measured at world 8: ~0.25 ms per os.link /
// os.replace / os.remove on the control loop, 0.8 ms per replica link of one output). These
// calls do a whole bundle's files per GIL release: the writer spools a bundle with one call,
// a replica links a bundle's files with one call.
//
// Reference: the replica side of SDFS PUTs (file_service.py:52-124, one scp per file).
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <string>

extern "C" {

// Write n files into directory `dir` (created if missing): dir/names[i] <- datas[i][0:lens[i]].
// Returns 0, or -errno of the first failure (files before it are written).
int dml_spool_write(const char* dir, int n, const char* const* names, const char* const* datas, const long* lens) {
  if (mkdir(dir, 0755) != 0 && errno != EEXIST) return -errno;
  std::string path;
  for (int i = 0; i < n; ++i) {
    if (std::strchr(names[i], '/')) return -EINVAL;
    path.assign(dir).append("/").append(names[i]);
    const int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (fd < 0) return -errno;
    long off = 0;
    while (off < lens[i]) {
      const ssize_t w = write(fd, datas[i] + off, (size_t)(lens[i] - off));
      if (w < 0) {
        if (errno == EINTR) continue;
        const int e = errno;
        close(fd);
        return -e;
      }
      off += w;
    }
    if (close(fd) != 0) return -errno;
  }
  return 0;
}

// For each i: make dsts[i] a hard link of srcs[i], atomically replacing an existing dsts[i]
// (link to dsts[i] + ".lnk", then rename). status[i] = 0 or -errno.
// Returns the number of files linked.
int dml_link_many(int n, const char* const* srcs, const char* const* dsts, int* status) {
  int ok = 0;
  std::string tmp;
  for (int i = 0; i < n; ++i) {
    tmp.assign(dsts[i]).append(".lnk");
    unlink(tmp.c_str());
    if (link(srcs[i], tmp.c_str()) != 0) {
      status[i] = -errno;
      continue;
    }
    if (rename(tmp.c_str(), dsts[i]) != 0) {
      status[i] = -errno;
      unlink(tmp.c_str());
      continue;
    }
    status[i] = 0;
    ++ok;
  }
  return ok;
}

// Read n whole files into one buffer: sizes first (pass buf = nullptr: lens[i] = size or
// -errno), then the bytes (buf of at least sum(lens) bytes, offs[i] = where file i starts).
// Returns the total size, or -errno of the first failure. The image store's local fast path:
// a window's 256 JPEGs in two GIL releases instead of one event-loop coroutine per file.
long dml_read_many(int n, const char* const* paths, char* buf, long cap, long* offs, long* lens) {
  if (!buf) {
    long total = 0;
    for (int i = 0; i < n; ++i) {
      struct stat st;
      if (stat(paths[i], &st) != 0) return -errno;
      lens[i] = (long)st.st_size;
      total += lens[i];
    }
    return total;
  }
  long off = 0;
  for (int i = 0; i < n; ++i) {
    if (off + lens[i] > cap) return -ENOSPC;
    const int fd = open(paths[i], O_RDONLY | O_CLOEXEC);
    if (fd < 0) return -errno;
    long got = 0;
    while (got < lens[i]) {
      const ssize_t r = read(fd, buf + off + got, (size_t)(lens[i] - got));
      if (r < 0) {
        if (errno == EINTR) continue;
        const int e = errno;
        close(fd);
        return -e;
      }
      if (r == 0) break;   // shrank since the stat: a short file
      got += r;
    }
    close(fd);
    offs[i] = off;
    lens[i] = got;
    off += got;
  }
  return off;
}

}  // extern "C"
