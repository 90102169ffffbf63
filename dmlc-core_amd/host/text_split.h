// text_split.h -- host-side text InputSplit with dmlc-core's chunk contract
// (InputSplit::Create(uri, part, nparts, "text"), src/io.cc:76-119):
//
//  * the input is a list of files built as InputSplitBase::InitInputFileInfo
//    does (input_split_base.cc:96-176): ';'-separated entries, each a file, a
//    directory (its entries in raw readdir order, dotfiles included, one
//    level) or a path whose last component is matched as a std::regex against
//    the directory's entries; empty files and directories dropped; no file at
//    all is an error;
//  * part k of n covers bytes [ceil(total/n)*k, ceil(total/n)*(k+1)) of the
//    concatenation, both ends moved forward to the next record start
//    (ResetPartition, input_split_base.cc:29-63; LineSplitter::SeekRecordBegin,
//    line_split.cc:11-36);
//  * chunks fill a read buffer (8 MiB by default, input_split_base.h:39) and are
//    cut after the last '\n' / '\r' in it (FindLastRecordBegin,
//    line_split.cc:37-45), the remainder carried into the next chunk; a record
//    longer than the buffer doubles it (Chunk::Load, input_split_base.cc:272-291);
//  * a '\n' is inserted after every file's last byte and at the end of input
//    when the last chunk would otherwise end mid-record (Read / ReadChunk,
//    input_split_base.cc:204-210, 247-254).
#pragma once
#include <cstdint>
#include <cstdio>
#include <string>
#include <utility>
#include <vector>

namespace dmlc_amd {

// A piece of a batch's text without a host copy (TextSplit::FillPieces): len
// bytes at src -- inside a file mapped by the split -- for batch offset off;
// src == nullptr: one inserted '\n'.
struct TextPiece {
  uint64_t off;
  const char *src;
  uint64_t len;
};

class TextSplit {
 public:
  TextSplit(const std::string &uri, unsigned part, unsigned nparts, size_t buffer_bytes = 8u << 20);
  ~TextSplit();
  TextSplit(const TextSplit &) = delete;
  TextSplit &operator=(const TextSplit &) = delete;

  // Appends the next chunk to *out; false at the end of the part.
  bool NextChunk(std::vector<char> *out);

  // In-place form for the device pipeline: reads whole chunks straight into
  // dst (capacity cap bytes) -- the same byte sequence and the same cuts as
  // NextChunk -- until at least max_bytes are filled or the next chunk might
  // not fit.  Each chunk's end offset (relative to dst) is appended to *ends.
  // The partial record after the last cut is kept for the next call.
  struct Fill {
    bool end;     // the part is exhausted
    size_t need;  // > 0: not even one chunk fits; call again with cap >= need
  };
  Fill FillChunks(char *dst, size_t cap, size_t max_bytes, std::vector<uint64_t> *ends);
  // The same chunks as pieces of the mapped files (no host copy): the batch's
  // text is the pieces in order, its chunk ends go to *ends as above, until
  // at least max_bytes are described.  Only when Mapped(); the two forms must
  // not be mixed between BeforeFirst calls.
  Fill FillPieces(size_t max_bytes, std::vector<uint64_t> *ends, std::vector<TextPiece> *pieces);
  // Every file mapped read-only (DMLC_AMD_MMAP unset or not "0", every file
  // regular and mappable): the mappings, for the caller to register with HIP.
  bool Mapped() const { return mapped_; }
  const std::vector<std::pair<const char *, size_t>> &Mappings() const { return maps_; }
  // Rewind to the start of the part.
  void BeforeFirst();
  // Bytes of this part's byte range consumed so far.
  size_t BytesRead() const { return offset_curr_ - offset_begin_; }
  // Bytes of the whole input (every part; InputSplit::GetTotalSize).
  uint64_t TotalSize() const { return offset_.back(); }

 private:
  size_t Read(char *buf, size_t size);
  void ReadAt(char *buf, size_t len, uint64_t pos);  // pread, split over threads when large
  uint64_t SeekRecordBegin(size_t file, uint64_t pos);
  size_t FileOf(uint64_t off) const;
  bool OpenAt(size_t file, uint64_t pos);

  std::vector<std::string> files_;
  std::vector<uint64_t> offset_;  // files_.size() + 1 prefix sums of the sizes
  uint64_t offset_begin_ = 0, offset_end_ = 0, offset_curr_ = 0;
  size_t file_ptr_ = 0;
  int fd_ = -1;
  uint64_t file_pos_ = 0;  // read position in files_[file_ptr_]
  size_t buffer_bytes_;
  std::vector<char> overflow_;  // partial record carried to the next chunk
  // mapped form: every file's mapping, and the carried partial record as pieces
  size_t ReadPieces(std::vector<TextPiece> *pv, uint64_t *size, size_t want);
  bool mapped_ = false;
  std::vector<std::pair<const char *, size_t>> maps_;
  std::vector<TextPiece> overflow_pieces_;
};

// Expand a URI path (file, directory or ';'-separated list) into file paths.
std::vector<std::string> ListInputFiles(const std::string &path);

}  // namespace dmlc_amd
