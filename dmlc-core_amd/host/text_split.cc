// text_split.cc -- see text_split.h for the contract and reference citations.
#include "text_split.h"

#include <dirent.h>
#include <sched.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <algorithm>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <regex>
#include <sstream>
#include <thread>

#include "dmlc/base.h"

namespace dmlc_amd {
namespace {

bool is_newline(char c) { return c == '\n' || c == '\r'; }

uint64_t file_size(const std::string &p) {
  struct stat st;
  if (stat(p.c_str(), &st) != 0) throw dmlc::Error("Check failed: file \"" + p + "\" does not exist");
  return (uint64_t)st.st_size;
}

// ---- the input file list, as InputSplitBase::InitInputFileInfo builds it
// (input_split_base.cc:96-176) over LocalFileSystem (local_filesys.cc:69-122)

struct PathInfo {
  std::string name;
  uint64_t size;
  bool dir;
};

// LocalFileSystem::GetPathInfo: stat; a dangling symlink (lstat only) is an
// empty file; anything else that cannot be stat'ed is fatal.
PathInfo GetPathInfo(const std::string &name) {
  struct stat sb;
  if (stat(name.c_str(), &sb) == -1) {
    const int errsv = errno;
    if (lstat(name.c_str(), &sb) == 0) return PathInfo{name, 0, false};
    throw dmlc::Error("LocalFileSystem.GetPathInfo: " + name + " error: " + std::strerror(errsv));
  }
  return PathInfo{name, (uint64_t)sb.st_size, S_ISDIR(sb.st_mode)};
}

// LocalFileSystem::ListDirectory: raw readdir order, every entry except "."
// and ".." (dotfiles included).
std::vector<PathInfo> ListDirectory(const std::string &dir) {
  DIR *d = opendir(dir.c_str());
  if (d == nullptr) {
    const int errsv = errno;
    throw dmlc::Error("LocalFileSystem.ListDirectory " + dir + " error: " + std::strerror(errsv));
  }
  std::vector<PathInfo> out;
  while (dirent *e = readdir(d)) {
    if (!std::strcmp(e->d_name, ".") || !std::strcmp(e->d_name, "..")) continue;
    std::string q = dir;
    if (q.empty() || q.back() != '/') q += '/';
    q += e->d_name;
    try {
      out.push_back(GetPathInfo(q));
    } catch (...) {
      closedir(d);
      throw;
    }
  }
  closedir(d);
  return out;
}

std::string StripEnd(std::string s, char c) {
  while (!s.empty() && s.back() == c) s.pop_back();
  return s;
}

// URI(path).name for the local file system (io.h:523-551): "file://host/p" -> "/p"
std::string LocalName(const std::string &u) {
  const size_t p = u.find("://");
  if (p == std::string::npos) return u;
  const std::string proto = u.substr(0, p + 3);
  if (proto != "file://") throw dmlc::Error("unsupported file system " + proto + " in \"" + u + "\" (local files only)");
  const size_t slash = u.find('/', p + 3);
  return slash == std::string::npos ? std::string("/") : u.substr(slash);
}

}  // namespace

std::vector<std::string> ListInputFiles(const std::string &uri) {
  // ConvertToURIs: split on ';' (std::getline semantics, common.h Split), then
  // per entry: a bare name or a name ending in '/' is taken as it is; else the
  // entry's directory is listed and an exact name match wins, otherwise every
  // non-empty file whose full path matches the entry as a std::regex
  std::vector<std::string> expanded;
  {
    std::istringstream is(uri);
    std::string item;
    while (std::getline(is, item, ';')) {
      const std::string name = LocalName(item);
      const size_t pos = name.rfind('/');
      if (pos == std::string::npos || pos + 1 == name.size()) {
        expanded.push_back(name);
        continue;
      }
      const std::vector<PathInfo> dfiles = ListDirectory(name.substr(0, pos));
      bool exact = false;
      for (const PathInfo &f : dfiles) {
        if (StripEnd(f.name, '/') == StripEnd(name, '/')) {
          expanded.push_back(f.name);
          exact = true;
          break;
        }
      }
      if (exact) continue;
      std::regex pattern;
      try {
        pattern = std::regex(name);
      } catch (const std::regex_error &e) {
        throw dmlc::Error(std::string(e.what()) + " bad regex " + name);
      }
      for (const PathInfo &f : dfiles) {
        if (f.dir || f.size == 0) continue;
        if (std::regex_match(StripEnd(f.name, '/'), pattern)) expanded.push_back(f.name);
      }
    }
  }
  // InitInputFileInfo: directories contribute their non-empty files (one
  // level, readdir order); empty files take no part
  std::vector<std::string> files;
  for (const std::string &path : expanded) {
    const PathInfo info = GetPathInfo(path);
    if (info.dir) {
      for (const PathInfo &f : ListDirectory(info.name))
        if (f.size != 0 && !f.dir) files.push_back(f.name);
    } else if (info.size != 0) {
      files.push_back(info.name);
    }
  }
  if (files.empty()) throw dmlc::Error("Check failed: files_.size() != 0U Cannot find any files that matches the URI pattern " + uri);
  return files;
}

TextSplit::TextSplit(const std::string &uri, unsigned part, unsigned nparts, size_t buffer_bytes)
    : buffer_bytes_(buffer_bytes) {
  if (nparts == 0 || part >= nparts) throw dmlc::Error("Check failed: part_index < num_parts");
  offset_.push_back(0);
  for (const std::string &f : ListInputFiles(uri)) {
    const uint64_t sz = file_size(f);
    if (sz == 0) continue;  // empty files take no part in the split
    files_.push_back(f);
    offset_.push_back(offset_.back() + sz);
  }
  // the mapped form (FillPieces): every file read-only mapped, unless
  // DMLC_AMD_MMAP=0 or a file cannot be (then every read is a pread)
  const char *mm = std::getenv("DMLC_AMD_MMAP");
  mapped_ = !(mm && mm[0] == '0') && !files_.empty();
  for (size_t i = 0; mapped_ && i < files_.size(); ++i) {
    const size_t sz = (size_t)(offset_[i + 1] - offset_[i]);
    const int fd = open(files_[i].c_str(), O_RDONLY);
    void *m = fd >= 0 ? mmap(nullptr, sz, PROT_READ, MAP_SHARED, fd, 0) : MAP_FAILED;
    if (fd >= 0) close(fd);
    if (m == MAP_FAILED) {
      mapped_ = false;
      break;
    }
    maps_.emplace_back((const char *)m, sz);
  }
  if (!mapped_) {
    for (auto &m : maps_) munmap(const_cast<char *>(m.first), m.second);
    maps_.clear();
  }
  const uint64_t total = offset_.back();
  const uint64_t step = (total + nparts - 1) / nparts;
  offset_begin_ = std::min(step * part, total);
  offset_end_ = std::min(step * (part + 1), total);
  if (offset_begin_ < offset_end_) {
    // move both ends to the next record start, within their files
    size_t fe = FileOf(offset_end_);
    if (offset_end_ != offset_[fe]) offset_end_ += SeekRecordBegin(fe, offset_end_ - offset_[fe]);
    size_t fb = FileOf(offset_begin_);
    if (offset_begin_ != offset_[fb]) offset_begin_ += SeekRecordBegin(fb, offset_begin_ - offset_[fb]);
  }
  BeforeFirst();
}

TextSplit::~TextSplit() {
  if (fd_ >= 0) close(fd_);
  for (auto &m : maps_) munmap(const_cast<char *>(m.first), m.second);
}

size_t TextSplit::FileOf(uint64_t off) const {
  size_t i = 0;
  while (i + 1 < offset_.size() && offset_[i + 1] <= off) ++i;
  return std::min(i, files_.empty() ? 0 : files_.size() - 1);
}

bool TextSplit::OpenAt(size_t file, uint64_t pos) {
  if (fd_ >= 0) close(fd_);
  fd_ = -1;
  if (file >= files_.size()) return false;
  fd_ = open(files_[file].c_str(), O_RDONLY);
  if (fd_ < 0) throw dmlc::Error("Check failed: cannot open \"" + files_[file] + "\"");
  file_pos_ = pos;
  return true;
}

// CPUs this process may use: its affinity mask, capped by a cgroup v2 CPU
// quota (cpu.max "quota period"; a GPU box's job gets a share of a large
// machine, whose processor count hardware_concurrency reports).
unsigned cpu_share() {
  unsigned n = std::max(1u, std::thread::hardware_concurrency());
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) n = std::min<unsigned>(n, std::max(1, (int)CPU_COUNT(&set)));
  if (FILE *f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    unsigned long long period = 0;
    if (std::fscanf(f, "%31s %llu", q, &period) == 2 && std::strcmp(q, "max") != 0 && period > 0) {
      const unsigned long long quota = std::strtoull(q, nullptr, 10);
      n = std::min<unsigned>(n, (unsigned)std::max<unsigned long long>(1, (quota + period - 1) / period));
    }
    std::fclose(f);
  }
  return n;
}

// Process-wide pool of reader threads (started once, never joined: no thread
// work at process exit).  ReadAt hands each a piece of a chunk; spawning and
// joining threads per 8 MiB chunk cost a fifth of the read time.
namespace {
class ReadPool {
 public:
  static ReadPool &get() {
    static ReadPool *p = new ReadPool();
    return *p;
  }
  size_t size() const { return nthreads_; }
  // run fn(0..n-1), piece 0 on the caller; rethrows the first error
  void run(size_t n, const std::function<void(size_t)> &fn) {
    std::unique_lock<std::mutex> job(job_mu_);  // one ReadAt at a time uses the pool
    std::string err;
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &fn;
      err_ = &err;
      next_ = 1;
      end_ = n;
      pending_ = n - 1;
      ++gen_;
    }
    cv_.notify_all();
    try {
      fn(0);
    } catch (const std::exception &e) {
      std::lock_guard<std::mutex> lk(mu_);
      if (err.empty()) err = e.what();
    }
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return pending_ == 0; });
    fn_ = nullptr;
    if (!err.empty()) throw dmlc::Error(err);
  }

 private:
  ReadPool() {
    const char *e = std::getenv("DMLC_AMD_READ_THREADS");
    nthreads_ = (size_t)std::min<unsigned>(e ? std::max(1, std::atoi(e)) : 8u, cpu_share());
    for (size_t i = 1; i < nthreads_; ++i) std::thread([this] { loop(); }).detach();
  }
  void loop() {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return gen_ != seen && next_ < end_; });
      seen = gen_;
      while (next_ < end_) {
        const size_t i = next_++;
        const std::function<void(size_t)> *fn = fn_;
        std::string *err = err_;
        lk.unlock();
        std::string what;
        try {
          (*fn)(i);
        } catch (const std::exception &e) {
          what = e.what();
        }
        lk.lock();
        if (!what.empty() && err->empty()) *err = what;
        if (--pending_ == 0) done_cv_.notify_all();
      }
    }
  }
  size_t nthreads_ = 1;
  std::mutex job_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(size_t)> *fn_ = nullptr;
  std::string *err_ = nullptr;
  size_t next_ = 0, end_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
};
}  // namespace

// len bytes of the open file at pos (all present: the size was taken at
// construction).  Large reads are split over the read pool: one core copies
// page cache at a fraction of what the host's memory system moves.
void TextSplit::ReadAt(char *buf, size_t len, uint64_t pos) {
  auto span = [this](char *b, size_t n, uint64_t at) {
    while (n) {
      const ssize_t r = pread(fd_, b, n, (off_t)at);
      if (r <= 0) throw dmlc::Error("Check failed: read of \"" + files_[file_ptr_] + "\"");
      b += r;
      n -= (size_t)r;
      at += (uint64_t)r;
    }
  };
  constexpr size_t kMinSplit = 1u << 20;
  ReadPool &pool = ReadPool::get();
  const size_t nt = std::min<size_t>(pool.size(), len / kMinSplit);
  if (nt <= 1) {
    span(buf, len, pos);
    return;
  }
  const size_t per = (len + nt - 1) / nt;
  pool.run(nt, [&](size_t i) {
    const size_t o = i * per;
    if (o < len) span(buf + o, std::min(per, len - o), pos + o);
  });
}

// Bytes from `pos` in `file` to the next record start: past the first newline
// run that follows pos (end of file if none).
uint64_t TextSplit::SeekRecordBegin(size_t file, uint64_t pos) {
  FILE *f = fopen(files_[file].c_str(), "rb");
  if (!f) throw dmlc::Error("Check failed: cannot open \"" + files_[file] + "\"");
  fseeko(f, (off_t)pos, SEEK_SET);
  uint64_t n = 0;
  int c;
  while ((c = fgetc(f)) != EOF) {
    ++n;
    if (is_newline((char)c)) break;
  }
  if (c != EOF) {
    while ((c = fgetc(f)) != EOF && is_newline((char)c)) ++n;
  }
  fclose(f);
  return n;
}

void TextSplit::BeforeFirst() {
  overflow_.clear();
  overflow_pieces_.clear();
  offset_curr_ = offset_begin_;
  if (offset_begin_ >= offset_end_ || files_.empty()) return;
  file_ptr_ = FileOf(offset_begin_);
  OpenAt(file_ptr_, offset_begin_ - offset_[file_ptr_]);
}

// Up to `size` bytes of the part; a '\n' follows each file's last byte.
size_t TextSplit::Read(char *buf, size_t size) {
  if (offset_begin_ >= offset_end_) return 0;
  if (offset_curr_ + size > offset_end_) size = offset_end_ - offset_curr_;
  if (size == 0) return 0;
  size_t left = size;
  while (fd_ >= 0) {
    const uint64_t remain = offset_[file_ptr_ + 1] - offset_[file_ptr_] - file_pos_;
    const size_t n = (size_t)std::min<uint64_t>(left, remain);
    if (n) ReadAt(buf, n, file_pos_);
    buf += n;
    left -= n;
    file_pos_ += n;
    offset_curr_ += n;
    if (left == 0) break;
    // end of this file: newline, then the next file
    *buf++ = '\n';
    --left;
    if (file_ptr_ + 1 >= files_.size()) break;
    OpenAt(++file_ptr_, 0);
  }
  return size - left;
}

bool TextSplit::NextChunk(std::vector<char> *out) {
  // the reference buffer is buffer_bytes/4 + 1 words with the last one a
  // sentinel; growing doubles the word count (Chunk::Load), so usable sizes run
  // B, 2B+4, 4B+12, ...
  size_t words = buffer_bytes_ / 4 + 1;
  for (;;) {
    const size_t cap = (words - 1) * 4;
    if (cap <= overflow_.size()) {  // a record longer than the buffer: grow it
      words *= 2;
      continue;
    }
    std::vector<char> buf(cap + 1);
    std::memcpy(buf.data(), overflow_.data(), overflow_.size());
    const size_t olen = overflow_.size();
    size_t n = Read(buf.data() + olen, cap - olen) + olen;
    if (n == 0) return false;
    if (n == olen) buf[n++] = '\n';  // end of input mid-record
    // cut after the last newline (the chunk keeps whole records)
    size_t cut = 0;
    for (size_t p = n - 1; p > 0; --p) {
      if (is_newline(buf[p])) {
        cut = p + 1;
        break;
      }
    }
    if (cut == 0) {  // no record boundary yet: keep reading with a bigger buffer
      overflow_.assign(buf.begin(), buf.begin() + n);
      words *= 2;
      continue;
    }
    out->insert(out->end(), buf.begin(), buf.begin() + cut);
    overflow_.assign(buf.begin() + cut, buf.begin() + n);
    return true;
  }
}

TextSplit::Fill TextSplit::FillChunks(char *dst, size_t cap, size_t max_bytes, std::vector<uint64_t> *ends) {
  size_t olen = overflow_.size();
  if (olen > cap) return Fill{false, olen + 1};
  std::memcpy(dst, overflow_.data(), olen);
  size_t pos = 0;  // start of the current chunk in dst
  Fill f{false, 0};
  while (pos < max_bytes) {
    size_t words = buffer_bytes_ / 4 + 1;  // as NextChunk: B, 2B+4, 4B+12, ...
    bool cut_made = false;
    for (;;) {
      const size_t C = (words - 1) * 4;
      if (C <= olen) {
        words *= 2;
        continue;
      }
      if (pos + C + 1 > cap) {  // the next chunk might not fit here
        if (pos == 0) f.need = C + 1;
        break;
      }
      size_t n = Read(dst + pos + olen, C - olen) + olen;
      if (n == 0) {
        f.end = true;
        break;
      }
      if (n == olen) dst[pos + n++] = '\n';  // end of input mid-record
      size_t cut = 0;
      for (size_t p = n - 1; p > 0; --p) {
        if (is_newline(dst[pos + p])) {
          cut = p + 1;
          break;
        }
      }
      if (cut == 0) {  // no record boundary yet: read on with a bigger buffer
        olen = n;
        words *= 2;
        continue;
      }
      pos += cut;
      olen = n - cut;
      ends->push_back(pos);
      cut_made = true;
      break;
    }
    if (!cut_made) break;
  }
  overflow_.assign(dst + pos, dst + pos + olen);
  return f;
}

// Read's walk over the files as pieces of their mappings (no copy): up to
// `want` bytes of the part appended to *pv at offset *size.
size_t TextSplit::ReadPieces(std::vector<TextPiece> *pv, uint64_t *size, size_t want) {
  if (offset_begin_ >= offset_end_) return 0;
  if (offset_curr_ + want > offset_end_) want = offset_end_ - offset_curr_;
  if (want == 0) return 0;
  size_t left = want;
  while (fd_ >= 0) {
    const uint64_t remain = offset_[file_ptr_ + 1] - offset_[file_ptr_] - file_pos_;
    const size_t n = (size_t)std::min<uint64_t>(left, remain);
    if (n) {
      const char *src = maps_[file_ptr_].first + file_pos_;
      if (!pv->empty() && pv->back().src && pv->back().src + pv->back().len == src) pv->back().len += n;
      else pv->push_back(TextPiece{*size, src, n});
      *size += n;
    }
    left -= n;
    file_pos_ += n;
    offset_curr_ += n;
    if (left == 0) break;
    pv->push_back(TextPiece{*size, nullptr, 1});  // end of this file: newline, then the next file
    *size += 1;
    --left;
    if (file_ptr_ + 1 >= files_.size()) break;
    OpenAt(++file_ptr_, 0);
  }
  return want - left;
}

namespace {
// the last '\n' / '\r' in batch bytes [lo, hi) of the pieces (hi if none)
uint64_t last_newline(const std::vector<TextPiece> &pv, uint64_t lo, uint64_t hi) {
  for (size_t i = pv.size(); i-- > 0;) {
    const TextPiece &p = pv[i];
    if (p.off >= hi) continue;
    if (p.off + p.len <= lo) break;
    const uint64_t a = std::max(p.off, lo), b = std::min(p.off + p.len, hi);
    if (!p.src) return a;  // an inserted newline (one byte)
    for (uint64_t x = b; x-- > a;) {
      const char c = p.src[x - p.off];
      if (c == '\n' || c == '\r') return x;
    }
  }
  return hi;
}
}  // namespace

// FillChunks over the mapped files: the same reads, cuts and carried
// remainder, with the bytes left where they are (pieces of the mappings).
TextSplit::Fill TextSplit::FillPieces(size_t max_bytes, std::vector<uint64_t> *ends, std::vector<TextPiece> *pv) {
  pv->clear();
  uint64_t size = 0;
  for (const TextPiece &p : overflow_pieces_) {
    pv->push_back(TextPiece{size, p.src, p.len});
    size += p.len;
  }
  size_t olen = (size_t)size;
  size_t pos = 0;
  Fill f{false, 0};
  while (pos < max_bytes) {
    size_t words = buffer_bytes_ / 4 + 1;  // as NextChunk: B, 2B+4, 4B+12, ...
    bool cut_made = false;
    for (;;) {
      const size_t C = (words - 1) * 4;
      if (C <= olen) {
        words *= 2;
        continue;
      }
      size_t n = ReadPieces(pv, &size, C - olen) + olen;
      if (n == 0) {
        f.end = true;
        break;
      }
      if (n == olen) {  // end of input mid-record
        pv->push_back(TextPiece{size, nullptr, 1});
        size += 1;
        ++n;
      }
      // cut after the last newline at chunk offset >= 1
      const uint64_t nl = last_newline(*pv, pos + 1, pos + n);
      if (nl == pos + n) {  // no record boundary yet: read on with a bigger buffer
        olen = n;
        words *= 2;
        continue;
      }
      const size_t cut = (size_t)(nl - pos) + 1;
      pos += cut;
      olen = n - cut;
      ends->push_back(pos);
      cut_made = true;
      break;
    }
    if (!cut_made) break;
  }
  // the remainder [pos, size) is carried as pieces; the batch keeps [0, pos)
  overflow_pieces_.clear();
  std::vector<TextPiece> keep;
  for (const TextPiece &p : *pv) {
    if (p.off < pos) {
      TextPiece q = p;
      if (q.off + q.len > pos) q.len = pos - q.off;
      keep.push_back(q);
    }
    if (p.off + p.len > pos) {
      const uint64_t a = std::max<uint64_t>(p.off, pos);
      overflow_pieces_.push_back(TextPiece{0, p.src ? p.src + (a - p.off) : nullptr, p.off + p.len - a});
    }
  }
  pv->swap(keep);
  return f;
}

}  // namespace dmlc_amd
