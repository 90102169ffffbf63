// io.cc -- dmlc/io.h for local files: InputSplit::Create(uri, part, nparts,
// "text") over TextSplit (text_split.h: the reference's chunk contract,
// src/io.cc:76-119, src/io/input_split_base.cc, src/io/line_split.cc) and
// Stream::Create for local files (src/io/local_filesys.cc:27-67).
#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "dmlc/io.h"
#include "dmlc/logging.h"
#include "dmlc_amd.h"
#include "text_split.h"

namespace dmlc_amd {
namespace {

std::string local_path(const char *uri) {
  std::string u = uri;
  if (u.compare(0, 7, "file://") == 0) u = u.substr(7);
  else if (u.find("://") != std::string::npos) LOG(FATAL) << "unsupported file system in \"" << uri << "\" (local files only)";
  return u;
}

// A local file opened with fopen (LocalFileSystem's FileStream).
class FileStream : public dmlc::SeekStream {
 public:
  FileStream(std::FILE *f, bool own) : f_(f), own_(own) {}
  ~FileStream() override {
    if (f_ && own_) std::fclose(f_);
  }
  size_t Read(void *ptr, size_t size) override { return std::fread(ptr, 1, size, f_); }
  void Write(const void *ptr, size_t size) override {
    CHECK(std::fwrite(ptr, 1, size, f_) == size) << "FileStream.Write incomplete";
  }
  void Seek(size_t pos) override { CHECK(fseeko(f_, (off_t)pos, SEEK_SET) == 0) << "FileStream.Seek failed"; }
  size_t Tell() override { return (size_t)ftello(f_); }

 private:
  std::FILE *f_;
  bool own_;
};

// InputSplit "text": whole chunks from TextSplit, records = lines.
class TextInputSplit : public dmlc::InputSplit {
 public:
  TextInputSplit(const std::string &uri, unsigned part, unsigned nparts)
      : uri_(uri), part_(part), nparts_(nparts), split_(new TextSplit(uri, part, nparts)) {}
  void HintChunkSize(size_t chunk_size) override {
    // the reference keeps the larger of the hint and its 8 MiB buffer (input_split_base.h:44-46)
    hint_ = std::max(hint_, chunk_size);
    split_.reset(new TextSplit(uri_, part_, nparts_, hint_));
  }
  size_t GetTotalSize() override { return split_->TotalSize(); }
  void BeforeFirst() override {
    split_->BeforeFirst();
    chunk_.clear();
    rec_ = 0;
  }
  bool NextChunk(Blob *out) override {
    chunk_.clear();
    rec_ = 0;
    if (!split_->NextChunk(&chunk_)) return false;
    out->dptr = chunk_.data();
    out->size = chunk_.size();
    return true;
  }
  // one line per record: the newline run after it is skipped (line_split.cc:47-72)
  bool NextRecord(Blob *out) override {
    for (;;) {
      while (rec_ < chunk_.size() && (chunk_[rec_] == '\n' || chunk_[rec_] == '\r')) ++rec_;
      if (rec_ < chunk_.size()) break;
      chunk_.clear();
      rec_ = 0;
      if (!split_->NextChunk(&chunk_)) return false;
    }
    size_t e = rec_;
    while (e < chunk_.size() && chunk_[e] != '\n' && chunk_[e] != '\r') ++e;
    out->dptr = chunk_.data() + rec_;
    out->size = e - rec_;
    if (e < chunk_.size()) chunk_[e] = '\0';
    rec_ = e + 1;
    return true;
  }
  void ResetPartition(unsigned part, unsigned nparts) override {
    part_ = part;
    nparts_ = nparts;
    split_.reset(new TextSplit(uri_, part, nparts, hint_));
    chunk_.clear();
    rec_ = 0;
  }

 private:
  std::string uri_;
  unsigned part_, nparts_;
  size_t hint_ = 8u << 20;
  std::unique_ptr<TextSplit> split_;
  std::vector<char> chunk_;
  size_t rec_ = 0;
};

}  // namespace
}  // namespace dmlc_amd

namespace dmlc {

Stream *Stream::Create(const char *uri, const char *const flag, bool allow_null) {
  const std::string path = dmlc_amd::local_path(uri);
  std::string mode = flag;
  if (mode == "r" || mode == "w" || mode == "a") mode += "b";
  std::FILE *f = (path == "stdin" && flag[0] == 'r') ? stdin : (path == "stdout" && flag[0] != 'r') ? stdout
                                                                                                  : std::fopen(path.c_str(), mode.c_str());
  if (f == nullptr) {
    if (allow_null) return nullptr;
    LOG(FATAL) << "LocalFileSystem::Open \"" << path << "\": " << std::strerror(errno);
  }
  return new dmlc_amd::FileStream(f, f != stdin && f != stdout);
}

SeekStream *SeekStream::CreateForRead(const char *uri, bool allow_null) {
  return static_cast<SeekStream *>(Stream::Create(uri, "r", allow_null));
}

InputSplit *InputSplit::Create(const char *uri, unsigned part_index, unsigned num_parts, const char *type) {
  CHECK(part_index < num_parts) << "invalid input parameter for InputSplit::Create";
  const std::string t = type;
  if (t != "text") LOG(FATAL) << "InputSplit type \"" << t << "\" is out of this build's scope (text only)";
  return new dmlc_amd::TextInputSplit(dmlc_amd::local_path(uri), part_index, num_parts);
}

}  // namespace dmlc

// ---- test hooks (C ABI): the InputSplit chunk sequence of a part, for
// tests/ to compare with the oracle on machines without a GPU.
extern "C" int dmlc_amd_host_split(const char *uri, unsigned part, unsigned nparts, uint64_t buffer_bytes,
                                   char **out_buf, uint64_t **out_off, uint64_t *out_n) {
  try {
    dmlc_amd::TextSplit split(uri, part, nparts, buffer_bytes);
    std::vector<char> all;
    std::vector<uint64_t> off(1, 0);
    while (split.NextChunk(&all)) off.push_back(all.size());
    *out_buf = static_cast<char *>(std::malloc(all.size() + 1));
    std::memcpy(*out_buf, all.data(), all.size());
    *out_off = static_cast<uint64_t *>(std::malloc(off.size() * 8));
    std::memcpy(*out_off, off.data(), off.size() * 8);
    *out_n = off.size() - 1;
    return 0;
  } catch (const std::exception &) {
    return DMLC_AMD_ERR_ARG;
  }
}

// Test hook: the same chunk sequence through TextSplit::FillChunks, the
// in-place reader of the device pipeline, with batches of batch_bytes into a
// buffer of cap bytes (small values exercise batch breaks and buffer growth).
extern "C" int dmlc_amd_host_split_inplace(const char *uri, unsigned part, unsigned nparts,
                                           uint64_t buffer_bytes, uint64_t batch_bytes, uint64_t cap,
                                           char **out_buf, uint64_t **out_off, uint64_t *out_n) {
  try {
    dmlc_amd::TextSplit split(uri, part, nparts, buffer_bytes);
    std::vector<char> all, buf(cap);
    std::vector<uint64_t> off(1, 0), ends;
    for (;;) {
      ends.clear();
      const dmlc_amd::TextSplit::Fill f = split.FillChunks(buf.data(), buf.size(), batch_bytes, &ends);
      if (f.need) {
        buf.resize(f.need);
        continue;
      }
      uint64_t prev = 0;
      for (uint64_t e : ends) {
        all.insert(all.end(), buf.data() + prev, buf.data() + e);
        off.push_back(all.size());
        prev = e;
      }
      if (f.end) break;
    }
    *out_buf = static_cast<char *>(std::malloc(all.size() + 1));
    std::memcpy(*out_buf, all.data(), all.size());
    *out_off = static_cast<uint64_t *>(std::malloc(off.size() * 8));
    std::memcpy(*out_off, off.data(), off.size() * 8);
    *out_n = off.size() - 1;
    return 0;
  } catch (const std::exception &) {
    return DMLC_AMD_ERR_ARG;
  }
}

// Test hook: the same chunk sequence through TextSplit::FillPieces (the
// mapped form: pieces of the files' mappings, DMA'd by the device pipeline),
// the bytes gathered from the pieces.  Fails (DMLC_AMD_ERR_ARG) when the
// split did not map its files.
extern "C" int dmlc_amd_host_split_pieces(const char *uri, unsigned part, unsigned nparts, uint64_t buffer_bytes,
                                          uint64_t batch_bytes, char **out_buf, uint64_t **out_off,
                                          uint64_t *out_n) {
  try {
    dmlc_amd::TextSplit split(uri, part, nparts, buffer_bytes);
    if (!split.Mapped()) return DMLC_AMD_ERR_ARG;
    std::vector<char> all;
    std::vector<uint64_t> off(1, 0), ends;
    std::vector<dmlc_amd::TextPiece> pv;
    for (;;) {
      ends.clear();
      const dmlc_amd::TextSplit::Fill f = split.FillPieces(batch_bytes, &ends, &pv);
      std::vector<char> batch;
      for (const dmlc_amd::TextPiece &pc : pv) {
        if (pc.off != batch.size()) return DMLC_AMD_ERR_ARG;  // pieces must tile the batch
        if (pc.src) batch.insert(batch.end(), pc.src, pc.src + pc.len);
        else batch.push_back('\n');
      }
      uint64_t prev = 0;
      for (uint64_t e : ends) {
        if (e > batch.size()) return DMLC_AMD_ERR_ARG;
        all.insert(all.end(), batch.data() + prev, batch.data() + e);
        off.push_back(all.size());
        prev = e;
      }
      if (prev != batch.size()) return DMLC_AMD_ERR_ARG;  // the batch is its chunks
      if (f.end) break;
    }
    *out_buf = static_cast<char *>(std::malloc(all.size() + 1));
    std::memcpy(*out_buf, all.data(), all.size());
    *out_off = static_cast<uint64_t *>(std::malloc(off.size() * 8));
    std::memcpy(*out_off, off.data(), off.size() * 8);
    *out_n = off.size() - 1;
    return 0;
  } catch (const std::exception &) {
    return DMLC_AMD_ERR_ARG;
  }
}

extern "C" void dmlc_amd_host_free(void *p) { std::free(p); }
