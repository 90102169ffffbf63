/*
 * dmlc/data.h -- the data-parser API of dmlc-core (include/dmlc/data.h in the
 * reference), provided by this build so downstream callers compile and link
 * against it unmodified.  The text parsers behind Parser<I,D>::Create run on
 * MI355X through the C ABI in dmlc_amd.h (dmlc-core_amd/host/hip_parser.cc).
 *
 * Surface kept from the reference:
 *   real_t / index_t                        data.h:27-29
 *   DataIter<T>                             data.h:56-67
 *   Row<I,D> and its accessors               data.h:74-163
 *   RowBlock<I,D> (CSR view, Slice)          data.h:175-247, 366-394
 *   RowBlockIter<I,D>::Create               data.h:264-282
 *   Parser<I,D>::Create / BytesRead          data.h:300-322
 * Instantiations: IndexType in {uint32_t, uint64_t}; DType in {float, int32_t,
 * int64_t} (CSV only for the integral ones), as registered by src/data.cc:202-221.
 */
#ifndef DMLC_DATA_H_
#define DMLC_DATA_H_

#include <cstddef>
#include <cstdint>
#include <string>

#include "dmlc/base.h"

namespace dmlc {

/*! \brief floating point type of labels and values */
typedef float real_t;
/*! \brief default feature index type */
typedef unsigned index_t;

/*! \brief pull-style iterator */
template <typename DType>
class DataIter {
 public:
  virtual ~DataIter() {}
  /*! \brief rewind to the beginning */
  virtual void BeforeFirst() = 0;
  /*! \brief advance; false at the end */
  virtual bool Next() = 0;
  /*! \brief the current item, valid until the next call to Next() */
  virtual const DType &Value() const = 0;
};

/*! \brief one sparse row (a view into a RowBlock) */
template <typename IndexType, typename DType = real_t>
class Row {
 public:
  const DType *label;
  const real_t *weight;
  const uint64_t *qid;
  size_t length;
  const IndexType *field;
  const IndexType *index;
  const DType *value;

  inline IndexType get_field(size_t i) const { return field[i]; }
  inline IndexType get_index(size_t i) const { return index[i]; }
  /*! \brief the i-th value; 1 when the row carries no values (binary features) */
  inline DType get_value(size_t i) const { return value == nullptr ? DType(1.0f) : value[i]; }
  inline DType get_label() const { return *label; }
  /*! \brief instance weight; 1 when absent */
  inline real_t get_weight() const { return weight == nullptr ? 1.0f : *weight; }
  /*! \brief query id; 0 when absent */
  inline uint64_t get_qid() const { return qid == nullptr ? 0 : *qid; }
  /*! \brief dot product with a dense weight vector (indices beyond it are skipped) */
  template <typename V>
  inline V SDot(const V *w, size_t size) const {
    V sum = static_cast<V>(0);
    for (size_t i = 0; i < length; ++i) {
      if (index[i] < size) sum += w[index[i]] * (value == nullptr ? V(1) : static_cast<V>(value[i]));
    }
    return sum;
  }
};

/*! \brief a block of rows in CSR form; every pointer is NULL when its array is empty */
template <typename IndexType, typename DType = real_t>
struct RowBlock {
  size_t size;              /*!< number of rows */
  const size_t *offset;     /*!< size + 1 entries; offset[0] may be non-zero */
  const DType *label;       /*!< size entries (NULL when there are no labels) */
  const real_t *weight;     /*!< size entries or NULL */
  const uint64_t *qid;      /*!< size entries or NULL */
  const IndexType *field;   /*!< libfm fields or NULL */
  const IndexType *index;   /*!< feature indices, addressed by offset[] */
  const DType *value;       /*!< feature values or NULL */

  inline Row<IndexType, DType> operator[](size_t rowid) const {
    Row<IndexType, DType> r;
    r.label = label + rowid;
    r.weight = weight == nullptr ? nullptr : weight + rowid;
    r.qid = qid == nullptr ? nullptr : qid + rowid;
    r.length = offset[rowid + 1] - offset[rowid];
    r.field = field == nullptr ? nullptr : field + offset[rowid];
    r.index = index + offset[rowid];
    r.value = value == nullptr ? nullptr : value + offset[rowid];
    return r;
  }
  /*! \brief bytes referenced by this block */
  inline size_t MemCostBytes() const {
    const size_t nnz = offset[size] - offset[0];
    size_t b = (size + 1) * sizeof(size_t) + nnz * sizeof(IndexType);
    if (label != nullptr) b += size * sizeof(DType);
    if (weight != nullptr) b += size * sizeof(real_t);
    if (qid != nullptr) b += size * sizeof(uint64_t);
    if (field != nullptr) b += nnz * sizeof(IndexType);
    if (value != nullptr) b += nnz * sizeof(DType);
    return b;
  }
  /*! \brief rows [begin, end) as a block of their own (pointers shared) */
  inline RowBlock Slice(size_t begin, size_t end) const {
    RowBlock r;
    r.size = end - begin;
    r.offset = offset + begin;
    r.label = label == nullptr ? nullptr : label + begin;
    r.weight = weight == nullptr ? nullptr : weight + begin;
    r.qid = qid == nullptr ? nullptr : qid + begin;
    r.field = field;
    r.index = index;
    r.value = value;
    return r;
  }
};

/*!
 * \brief iterator over the whole dataset as RowBlocks; Create() loads the
 * dataset into memory (the reference's BasicRowIter, src/data/basic_row_iter.h).
 */
template <typename IndexType, typename DType = real_t>
class RowBlockIter : public DataIter<RowBlock<IndexType, DType> > {
 public:
  static RowBlockIter<IndexType, DType> *Create(const char *uri, unsigned part_index, unsigned num_parts,
                                                const char *type);
  /*! \brief 1 + the largest feature index seen */
  virtual size_t NumCol() const = 0;
};

/*!
 * \brief parser of text formats ("libsvm", "csv", or "auto" with a format=
 * URI argument) into RowBlocks.  uri: file, directory or ';'-separated list,
 * optionally followed by ?key=value&... parser arguments.  part_index /
 * num_parts select a byte range of the input (data-parallel sharding).
 */
template <typename IndexType, typename DType = real_t>
class Parser : public DataIter<RowBlock<IndexType, DType> > {
 public:
  static Parser<IndexType, DType> *Create(const char *uri, unsigned part_index, unsigned num_parts,
                                          const char *type);
  /*! \brief bytes of input consumed so far */
  virtual size_t BytesRead() const = 0;
};

}  // namespace dmlc

#endif  // DMLC_DATA_H_
