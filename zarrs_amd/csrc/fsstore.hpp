// Filesystem store reads for the decode call (host ingestion).
//
// Mirrors zarrs_filesystem's FilesystemStore read side:
//  * key -> path is the caller's (FilesystemStore::key_to_fspath, zarrs_filesystem/src/lib.rs:173-179);
//  * a missing file is a missing key (Ok(None) -> fill value, lib.rs:339-343, 428-430);
//  * a byte range past the end of the file is an InvalidByteRangeError (lib.rs:437-447, 375-382);
//  * buffered reads are positional (read_exact_at, lib.rs:452-459); with direct I/O the pages a
//    range intersects are read with O_DIRECT into page-aligned memory and the range is sliced out
//    (get_partial_many_direct_io + coalesce_byte_ranges_with_page_size, lib.rs:323-415,
//    direct_io.rs:25-50).
// Here the destination is pinned (page-locked) staging memory that is DMA'd to HBM, and the reads
// of one sub-batch run on a pool of host threads while the previous sub-batch is copied and decoded.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace zgpu {

struct FileRange {
  const char *path = nullptr;  // NULL: missing key
  uint64_t offset = 0;
  uint64_t len = 0;            // UINT64_MAX: to the end of the file
  // resolved by fs_open_all
  int fd = -1;
  bool direct = false;         // opened with O_DIRECT
  bool missing = true;         // no such file (or path NULL)
  bool bad_range = false;      // range beyond the end of the file
  uint64_t size = 0;           // file size
  uint64_t rd_off = 0, rd_len = 0;  // what is read (page-aligned under O_DIRECT)
  uint64_t slab_off = 0;       // where the read lands in its sub-batch's staging slab
};

// Open + fstat every range on `threads` host threads; resolves missing / bad_range / rd_*.
// Returns "" or the first hard I/O error (permission denied, EIO, ...).
std::string fs_open_all(std::vector<FileRange> &r, bool direct_io, int threads);
// Read ranges r[idx[k]] into slab + r[.].slab_off on `threads` host threads. Returns "" or an error.
std::string fs_read_into(std::vector<FileRange> &r, const std::vector<uint64_t> &idx, uint8_t *slab, int threads);
void fs_close_all(std::vector<FileRange> &r);

}  // namespace zgpu
