/*
 * dmlc/data.h -- dmlc-core's data-parser API (reference include/dmlc/data.h),
 * provided by this build so downstream callers compile and link against it
 * unchanged.  The text parsers registered here ("libsvm", "csv", "libfm";
 * dmlc-core_amd/host/data.cc) run on MI355X through the C ABI of
 * dmlc_amd.h.
 *
 * Surface (with the reference's semantics, citing reference data.h):
 *   real_t / index_t                          :27-34
 *   DataIter<T>                               :56-67
 *   Row<I,D>: accessors, SDot (CHECKs the
 *     index bound)                            :74-163
 *   RowBlock<I,D>: CSR view, operator[] and
 *     Slice (CHECKed), MemCostBytes           :175-247, :366-394
 *   RowBlockIter<I,D>::Create / NumCol        :264-282
 *   Parser<I,D>::Create / BytesRead / Factory :300-322
 *   ParserFactoryReg, DMLC_REGISTER_DATA_PARSER :329-363
 * Instantiated for IndexType in {uint32_t, uint64_t} and DType in {real_t,
 * int32_t, int64_t}, as src/data.cc:189-221 registers them.
 */
#ifndef DMLC_DATA_H_
#define DMLC_DATA_H_

#include <cstddef>
#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "./base.h"
#include "./io.h"
#include "./logging.h"
#include "./registry.h"

// lets a template argument list with a comma pass through a macro argument
#define __DMLC_COMMA ,

namespace dmlc {

/*! \brief floating point type of labels and values */
typedef float real_t;
/*! \brief default feature index type */
typedef unsigned index_t;

/*! \brief pull-style iterator: BeforeFirst(); while (Next()) use(Value()); */
template <typename DType>
class DataIter {
 public:
  virtual ~DataIter(void) DMLC_THROW_EXCEPTION {}
  /*! \brief rewind to the beginning */
  virtual void BeforeFirst(void) = 0;
  /*! \brief advance; false at the end */
  virtual bool Next(void) = 0;
  /*! \brief the current item, valid until the next call to Next() */
  virtual const DType &Value(void) const = 0;
};

/*! \brief one sparse row: a view into a RowBlock */
template <typename IndexType, typename DType = real_t>
class Row {
 public:
  const DType *label;     /*!< label of the row */
  const real_t *weight;   /*!< instance weight, or NULL */
  const uint64_t *qid;    /*!< query / session id, or NULL */
  size_t length;          /*!< number of entries */
  const IndexType *field; /*!< field of each entry (libfm), or NULL */
  const IndexType *index; /*!< feature index of each entry */
  const DType *value;     /*!< value of each entry, or NULL: every value is 1 */

  inline IndexType get_field(size_t i) const { return field[i]; }
  inline IndexType get_index(size_t i) const { return index[i]; }
  inline DType get_value(size_t i) const { return value == nullptr ? DType(1.0f) : value[i]; }
  inline DType get_label() const { return *label; }
  inline real_t get_weight() const { return weight == nullptr ? 1.0f : *weight; }
  inline uint64_t get_qid() const { return qid == nullptr ? 0 : *qid; }
  /*! \brief sum of weight[index[i]] * value[i]; an index >= size is a fatal error */
  template <typename V>
  inline V SDot(const V *weight, size_t size) const {
    V sum = static_cast<V>(0);
    for (size_t i = 0; i < length; ++i) {
      CHECK(index[i] < size) << "feature index exceed bound";
      sum += value == nullptr ? weight[index[i]] : weight[index[i]] * value[i];
    }
    return sum;
  }
};

/*!
 * \brief a block of rows in CSR form.  Row r's entries are
 * [offset[r], offset[r+1]) of index / field / value; blocks handed out by a
 * Parser start at offset[0] == 0 (a Slice may not).  weight / qid / field /
 * value are NULL when the block carries none.
 */
template <typename IndexType, typename DType = real_t>
struct RowBlock {
  size_t size;              /*!< number of rows */
  const size_t *offset;     /*!< size + 1 row pointers */
  const DType *label;       /*!< size labels */
  const real_t *weight;     /*!< size weights or NULL */
  const uint64_t *qid;      /*!< size query ids or NULL */
  const IndexType *field;   /*!< field ids or NULL */
  const IndexType *index;   /*!< feature indices */
  const DType *value;       /*!< feature values or NULL */

  /*! \brief row rowid (CHECKs rowid < size) */
  inline Row<IndexType, DType> operator[](size_t rowid) const;
  /*! \brief bytes of the block's arrays, counted as the reference counts them */
  inline size_t MemCostBytes(void) const {
    size_t cost = size * (sizeof(size_t) + sizeof(DType));
    if (weight != nullptr) cost += size * sizeof(real_t);
    if (qid != nullptr) cost += size * sizeof(size_t);
    const size_t ndata = offset[size] - offset[0];
    if (field != nullptr) cost += ndata * sizeof(IndexType);
    if (index != nullptr) cost += ndata * sizeof(IndexType);
    if (value != nullptr) cost += ndata * sizeof(DType);
    return cost;
  }
  /*! \brief rows [begin, end) sharing this block's arrays (CHECKs the range) */
  inline RowBlock Slice(size_t begin, size_t end) const {
    CHECK(begin <= end && end <= size);
    RowBlock r;
    r.size = end - begin;
    r.label = label + begin;
    r.weight = weight == nullptr ? nullptr : weight + begin;
    r.qid = qid == nullptr ? nullptr : qid + begin;
    r.offset = offset + begin;
    r.field = field;
    r.index = index;
    r.value = value;
    return r;
  }
};

/*!
 * \brief the whole dataset as RowBlocks, held in memory (Create returns the
 * reference's BasicRowIter: every block of a Parser concatenated into one).
 */
template <typename IndexType, typename DType = real_t>
class RowBlockIter : public DataIter<RowBlock<IndexType, DType>> {
 public:
  /*! \brief load uri (see Parser::Create for uri, part_index, num_parts and type) */
  static RowBlockIter<IndexType, DType> *Create(const char *uri, unsigned part_index, unsigned num_parts,
                                                const char *type);
  /*! \brief largest feature index + 1 */
  virtual size_t NumCol() const = 0;
};

/*!
 * \brief parser of an input into RowBlocks.  uri: a file, a directory, a
 * ';'-separated list or a regex over a directory, then optionally
 * ?key=value&... parser arguments; part_index / num_parts select a byte range
 * of the input (data-parallel sharding).  type: a registered parser name
 * ("libsvm", "csv", "libfm") or "auto" (the uri's format= argument, else
 * libsvm).
 */
template <typename IndexType, typename DType = real_t>
class Parser : public DataIter<RowBlock<IndexType, DType>> {
 public:
  static Parser<IndexType, DType> *Create(const char *uri_, unsigned part_index, unsigned num_parts,
                                          const char *type);
  /*! \brief bytes of input consumed so far */
  virtual size_t BytesRead(void) const = 0;
  /*! \brief signature of a registered parser factory */
  typedef Parser<IndexType, DType> *(*Factory)(const std::string &path,
                                               const std::map<std::string, std::string> &args,
                                               unsigned part_index, unsigned num_parts);
};

/*! \brief registry entry of a parser factory */
template <typename IndexType, typename DType = real_t>
struct ParserFactoryReg
    : public FunctionRegEntryBase<ParserFactoryReg<IndexType, DType>, typename Parser<IndexType, DType>::Factory> {};

/*!
 * \brief register a parser factory under TypeName for Parser<IndexType, DataType>:
 *   DMLC_REGISTER_DATA_PARSER(uint32_t, real_t, mytype, CreateMyParser<uint32_t>);
 * after which Parser<uint32_t>::Create(uri, part, nparts, "mytype") calls it.
 */
#define DMLC_REGISTER_DATA_PARSER(IndexType, DataType, TypeName, FactoryFunction) \
  DMLC_REGISTRY_REGISTER(::dmlc::ParserFactoryReg<IndexType __DMLC_COMMA DataType>,  \
                         ParserFactoryReg##_##IndexType##_##DataType, TypeName)   \
      .set_body(FactoryFunction)

template <typename IndexType, typename DType>
inline Row<IndexType, DType> RowBlock<IndexType, DType>::operator[](size_t rowid) const {
  CHECK(rowid < size);
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

}  // namespace dmlc

#endif  // DMLC_DATA_H_
