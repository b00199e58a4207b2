// ct_format.hpp -- on-disk formats the GPU worker group reads and writes.
//
// herdsman stores client data as opaque rows and keys as opaque blobs:
//   * partition file <storage>/<session>/<frame>/<partition> = sequence of
//     rows, each `uint32 length` + payload        (/root/reference/src/service/storage_service.cpp:19-28,233-240)
//   * key file <key_dir>/<session>/<int(schema)>.key, written verbatim
//                                                  (/root/reference/src/service/key_service.cpp:19-44)
// Their payload encoding (presumably OpenFHE serialisation) is not pinned by
// anything in the tree, so this backend defines its own, documented in
// INTEGRATION.md:
//   row payload   = 1..k ciphertexts, each: CtHeader + 2*L*N u64 words
//   key file      = KeyFileHeader + n_keys x (KeyEntryHeader + dnum*2*(L+K)*N u64)
// All integers little-endian.
#pragma once
#include <cstdint>
#include <filesystem>
#include <string>
#include <vector>

namespace herdsman_gpu {

constexpr uint32_t kCtMagic = 0x54434648;   // "HFCT"
constexpr uint32_t kKeyMagic = 0x424B4648;  // "HFKB"

struct CtHeader {
  uint32_t magic = kCtMagic;
  uint16_t version = 1;
  uint8_t scheme = 0;   // 0 CKKS, 1 BFV
  uint8_t domain = 0;   // 1 = NTT (CKKS), 0 = coefficient (BFV)
  uint32_t log_n = 0;
  uint32_t n_limbs = 0; // L
  uint64_t moduli_digest = 0;  // FNV-1a of the Q moduli, guards against parameter mix-ups
};
static_assert(sizeof(CtHeader) == 24, "CtHeader layout");

struct KeyFileHeader {
  uint32_t magic = kKeyMagic;
  uint16_t version = 1;
  uint8_t scheme = 0;
  uint8_t pad = 0;
  uint32_t log_n = 0, L = 0, K = 0, dnum = 0, n_keys = 0, pad2 = 0;
  uint64_t moduli_digest = 0;  // FNV-1a of Q u P
};
static_assert(sizeof(KeyFileHeader) == 40, "KeyFileHeader layout");

struct KeyEntryHeader {
  uint32_t kind = 0;        // 0 = relinearisation, 1 = Galois
  uint32_t galois_elt = 0;  // for kind 1
};

uint64_t moduli_digest(const uint64_t *moduli, uint32_t count);

// rows of a partition file (payload bytes only)
std::vector<std::vector<uint8_t>> read_partition(const std::filesystem::path &path);
void write_partition(const std::filesystem::path &path, const std::vector<std::vector<uint8_t>> &rows);

// A partition file mapped read-only: rows are views into the mapping (no
// per-row allocation or copy; the worker stages them straight into pinned
// memory).  Throws on a missing file or a truncated row.
class PartitionView {
 public:
  explicit PartitionView(const std::filesystem::path &path);
  ~PartitionView();
  PartitionView(const PartitionView &) = delete;
  PartitionView &operator=(const PartitionView &) = delete;
  size_t size() const { return rows_.size(); }
  const uint8_t *row(size_t i) const { return rows_[i].first; }
  uint32_t row_len(size_t i) const { return rows_[i].second; }

 private:
  void *map_ = nullptr;
  size_t bytes_ = 0;
  std::vector<std::pair<const uint8_t *, uint32_t>> rows_;
};

// A partition file read with pread: the row index (payload offsets and
// lengths) is built once from the u32 length prefixes, and a caller reads any
// byte range of a row straight into its own memory (the worker's pinned
// staging buffers: one copy from the page cache, no mapping).  Throws on a
// missing file, a truncated row or a short read.
class PartitionIndex {
 public:
  explicit PartitionIndex(const std::filesystem::path &path);
  ~PartitionIndex();
  PartitionIndex(const PartitionIndex &) = delete;
  PartitionIndex &operator=(const PartitionIndex &) = delete;
  size_t size() const { return rows_.size(); }
  uint32_t row_len(size_t i) const { return rows_[i].second; }
  // bytes [off, off + len) of row i's payload -> dst
  void read(size_t i, size_t off, void *dst, size_t len) const;

 private:
  std::filesystem::path path_;
  int fd_ = -1;
  std::vector<std::pair<uint64_t, uint32_t>> rows_;  // payload file offset, length
};

// Output partition written through a temporary file renamed into place by
// commit(): a task that fails half-way leaves no output behind.  Rows are
// gathered with writev from caller memory (header + words), no staging copy.
// Like herdsman's own partition writes (storage_service.cpp), this protects
// against failures of the process; `durable` adds fsync of the file before
// the rename and of the directory after it, for a crash of the machine.
class PartitionWriter {
 public:
  explicit PartitionWriter(const std::filesystem::path &path, bool durable = false);
  ~PartitionWriter();
  PartitionWriter(const PartitionWriter &) = delete;
  PartitionWriter &operator=(const PartitionWriter &) = delete;
  // one row = `parts` byte ranges, written as u32 length + the ranges
  void append(const std::vector<std::pair<const void *, size_t>> &parts);
  // rows written in parallel: claim() reserves `bytes` at the end of the file
  // (one thread), write_row_at() writes one row (u32 length + parts) at a
  // claimed offset; calls on disjoint ranges may run concurrently
  uint64_t claim(uint64_t bytes);
  void write_row_at(uint64_t off, const std::vector<std::pair<const void *, size_t>> &parts) const;
  void commit();

 private:
  std::filesystem::path path_, tmp_;
  uint64_t end_ = 0;
  int fd_ = -1;
  bool done_ = false, durable_ = false;
};

}  // namespace herdsman_gpu
