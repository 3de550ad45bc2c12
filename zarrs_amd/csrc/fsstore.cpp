// Filesystem store reads (positional, optionally O_DIRECT) into pinned staging; see fsstore.hpp.
#include "fsstore.hpp"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstring>
#include <mutex>
#include <thread>

namespace zgpu {

static constexpr uint64_t kPage = 4096;
static constexpr uint64_t kPiece = 4ull << 20;  // read granule handed to a thread (page multiple)

template <class F>
static void run_pool(int threads, uint64_t n_tasks, F f) {
  if (threads <= 1 || n_tasks <= 1) {
    for (uint64_t i = 0; i < n_tasks; i++) f(i);
    return;
  }
  std::atomic<uint64_t> next{0};
  std::vector<std::thread> pool;
  const int nt = (int)std::min<uint64_t>((uint64_t)threads, n_tasks);
  pool.reserve(nt);
  for (int t = 0; t < nt; t++)
    pool.emplace_back([&] {
      for (uint64_t i; (i = next.fetch_add(1)) < n_tasks;) f(i);
    });
  for (auto &th : pool) th.join();
}

std::string fs_open_all(std::vector<FileRange> &r, bool direct_io, int threads) {
  std::mutex mu;
  std::string err;
  run_pool(threads, r.size(), [&](uint64_t i) {
    FileRange &f = r[i];
    f.missing = true;
    if (!f.path) return;
    int fd;
    f.direct = false;
    if (direct_io) {
      fd = ::open(f.path, O_RDONLY | O_CLOEXEC | O_DIRECT);
      if (fd >= 0) f.direct = true;
      else if (errno == EINVAL) fd = ::open(f.path, O_RDONLY | O_CLOEXEC);  // no O_DIRECT here (tmpfs)
    } else {
      fd = ::open(f.path, O_RDONLY | O_CLOEXEC);
    }
    if (fd < 0) {
      if (errno == ENOENT || errno == ENOTDIR) return;  // missing key
      std::lock_guard<std::mutex> lk(mu);
      if (err.empty()) err = std::string("open ") + f.path + ": " + std::strerror(errno);
      return;
    }
    struct stat st;
    if (::fstat(fd, &st) != 0) {
      std::lock_guard<std::mutex> lk(mu);
      if (err.empty()) err = std::string("fstat ") + f.path + ": " + std::strerror(errno);
      ::close(fd);
      return;
    }
    f.fd = fd;
    f.missing = false;
    f.size = (uint64_t)st.st_size;
    if (f.len == UINT64_MAX) {  // ByteRange::FromStart(offset, None)
      if (f.offset > f.size) f.bad_range = true;
      else f.len = f.size - f.offset;
    } else if (f.offset > f.size || f.len > f.size - f.offset) {
      f.bad_range = true;
    }
    if (f.bad_range) {
      f.len = 0;
      return;
    }
    if (f.direct) {  // the pages the range intersects
      f.rd_off = f.offset / kPage * kPage;
      f.rd_len = ((f.offset + f.len + kPage - 1) / kPage * kPage) - f.rd_off;
    } else {
      f.rd_off = f.offset;
      f.rd_len = f.len;
    }
  });
  return err;
}

std::string fs_read_into(std::vector<FileRange> &r, const std::vector<uint64_t> &idx, uint8_t *slab, int threads) {
  struct Piece { uint64_t range, off, len; };
  std::vector<Piece> pieces;
  for (uint64_t i : idx) {
    const FileRange &f = r[i];
    if (f.missing || f.bad_range || !f.rd_len) continue;
    for (uint64_t o = 0; o < f.rd_len; o += kPiece) pieces.push_back(Piece{i, o, std::min(kPiece, f.rd_len - o)});
  }
  std::mutex mu;
  std::string err;
  run_pool(threads, pieces.size(), [&](uint64_t k) {
    const Piece &p = pieces[k];
    const FileRange &f = r[p.range];
    uint8_t *dst = slab + f.slab_off + p.off;
    uint64_t done = 0;
    while (done < p.len) {
      const uint64_t pos = f.rd_off + p.off + done;
      const ssize_t n = ::pread(f.fd, dst + done, p.len - done, (off_t)pos);
      if (n < 0) {
        if (errno == EINTR) continue;
        std::lock_guard<std::mutex> lk(mu);
        if (err.empty()) err = std::string("read ") + f.path + ": " + std::strerror(errno);
        return;
      }
      if (n == 0 || pos + (uint64_t)n >= f.size) {  // end of file (O_DIRECT reads whole pages past it)
        if (pos + (uint64_t)n < f.offset + f.len) {
          std::lock_guard<std::mutex> lk(mu);
          if (err.empty()) err = std::string("read ") + f.path + ": file shrank while reading";
        }
        return;
      }
      done += (uint64_t)n;
    }
  });
  return err;
}

void fs_close_all(std::vector<FileRange> &r) {
  for (FileRange &f : r)
    if (f.fd >= 0) {
      ::close(f.fd);
      f.fd = -1;
    }
}

}  // namespace zgpu
