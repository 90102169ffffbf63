/*
 * dmlc/io.h -- the I/O interfaces the parse path touches (this build's own
 * header, API-compatible with the reference's include/dmlc/io.h):
 *
 *   Stream      byte stream with the reference's binary serialisation of
 *               PODs, strings and vectors (serializer.h: a vector is its
 *               element count as uint64 then the raw elements, little
 *               endian) -- the page format of RowBlockContainer::Save/Load
 *               (src/data/row_block.h:190-216)
 *   InputSplit  the chunk contract the text parsers consume (io.h:154-291):
 *               NextChunk hands over whole records only, its memory valid
 *               until the next call; Create(uri, part, nparts, "text")
 *               partitions the input by byte range as ResetPartition does.
 *
 * Local files only (the remote file systems are out of scope).
 */
#ifndef DMLC_IO_H_
#define DMLC_IO_H_

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "./base.h"
#include "./logging.h"

namespace dmlc {

/*! \brief interface of a byte stream */
class Stream {
 public:
  /*! \brief read up to size bytes; returns the bytes read (0 at the end) */
  virtual size_t Read(void *ptr, size_t size) = 0;
  /*! \brief write size bytes */
  virtual void Write(const void *ptr, size_t size) = 0;
  virtual ~Stream() DMLC_THROW_EXCEPTION {}
  /*!
   * \brief open a local file ("file://" prefix optional); flag "r", "w" or "a".
   * With allow_null a missing file for reading returns NULL instead of raising.
   */
  static Stream *Create(const char *uri, const char *const flag, bool allow_null = false);

  /*! \brief serialise one value: arithmetic, std::string or std::vector of arithmetic */
  template <typename T>
  inline void Write(const T &data);
  /*! \brief deserialise one value written by Write; false at the end of the stream */
  template <typename T>
  inline bool Read(T *out_data);
};

/*! \brief a stream that can seek (local files for reading) */
class SeekStream : public Stream {
 public:
  virtual void Seek(size_t pos) = 0;
  virtual size_t Tell(void) = 0;
  static SeekStream *CreateForRead(const char *uri, bool allow_null = false);
};

namespace io_detail {
template <typename T>
struct Pod {
  static_assert(std::is_arithmetic<T>::value, "Stream serialises arithmetic types, strings and vectors of them");
  static void Write(Stream *s, const T &v) { s->Write(&v, sizeof(T)); }
  static bool Read(Stream *s, T *v) { return s->Read(v, sizeof(T)) == sizeof(T); }
};
template <typename T>
struct Pod<std::vector<T>> {
  static void Write(Stream *s, const std::vector<T> &v) {
    static_assert(std::is_arithmetic<T>::value, "vectors of arithmetic types only");
    const uint64_t n = v.size();
    s->Write(&n, sizeof(n));
    if (n) s->Write(v.data(), sizeof(T) * v.size());
  }
  static bool Read(Stream *s, std::vector<T> *v) {
    uint64_t n = 0;
    if (s->Read(&n, sizeof(n)) != sizeof(n)) return false;
    v->resize((size_t)n);
    if (n == 0) return true;
    const size_t bytes = sizeof(T) * (size_t)n;
    return s->Read(v->data(), bytes) == bytes;
  }
};
template <>
struct Pod<std::string> {
  static void Write(Stream *s, const std::string &v) {
    const uint64_t n = v.size();
    s->Write(&n, sizeof(n));
    if (n) s->Write(v.data(), v.size());
  }
  static bool Read(Stream *s, std::string *v) {
    uint64_t n = 0;
    if (s->Read(&n, sizeof(n)) != sizeof(n)) return false;
    v->resize((size_t)n);
    return n == 0 || s->Read(&(*v)[0], (size_t)n) == (size_t)n;
  }
};
}  // namespace io_detail

template <typename T>
inline void Stream::Write(const T &data) {
  io_detail::Pod<T>::Write(this, data);
}
template <typename T>
inline bool Stream::Read(T *out_data) {
  return io_detail::Pod<T>::Read(this, out_data);
}

/*!
 * \brief input split: the input (a file, a directory, a ';'-separated list
 * or a regex over a directory's entries) cut into part_index of num_parts by
 * byte range, handed out as chunks of whole records.
 */
class InputSplit {
 public:
  /*! \brief a span of memory owned by the split */
  struct Blob {
    void *dptr;
    size_t size;
  };
  /*! \brief hint for the chunk buffer size in bytes (the default is 8 MiB) */
  virtual void HintChunkSize(size_t /*chunk_size*/) {}
  /*! \brief total bytes of the input (all parts) */
  virtual size_t GetTotalSize(void) = 0;
  /*! \brief rewind to the start of this part */
  virtual void BeforeFirst(void) = 0;
  /*! \brief next record (one line, without its newline); false at the end */
  virtual bool NextRecord(Blob *out_rec) = 0;
  /*! \brief next chunk of whole records; false at the end; valid until the next call */
  virtual bool NextChunk(Blob *out_chunk) = 0;
  /*! \brief chunk of about n_records records (text splits: one chunk) */
  virtual bool NextBatch(Blob *out_chunk, size_t /*n_records*/) { return NextChunk(out_chunk); }
  virtual ~InputSplit(void) DMLC_THROW_EXCEPTION {}
  /*! \brief move to another part of the same input */
  virtual void ResetPartition(unsigned part_index, unsigned num_parts) = 0;
  /*!
   * \brief create a split of `uri`; type "text" (one record per line).
   * Other types of the reference (recordio, indexed_recordio) stay out of
   * this build's scope and raise.
   */
  static InputSplit *Create(const char *uri, unsigned part_index, unsigned num_parts, const char *type);
};

}  // namespace dmlc

#endif  // DMLC_IO_H_
