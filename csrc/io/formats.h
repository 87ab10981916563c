// Header parsers of the two MNIST storage formats, free of Python/pybind11 so that the same code
// is linked into the ``_io`` extension AND into a standalone sanitizer/fuzz driver
// (csrc/io/fuzz_headers.cpp, built with -fsanitize=address,undefined by tests/test_io_fuzz.py).
//
// Every length read from a file is untrusted: additions and multiplications of header values are
// overflow-checked, and every byte range is checked against the buffer / file size before use.
#pragma once
#include <cstdint>
#include <limits>
#include <stdexcept>
#include <string>
#include <vector>

namespace mnist_io {

static inline uint32_t be32(const uint8_t* p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | uint32_t(p[3]);
}
static inline uint64_t be64(const uint8_t* p) { return (uint64_t(be32(p)) << 32) | be32(p + 4); }

// a * b, throwing instead of wrapping
static inline uint64_t mul_checked(uint64_t a, uint64_t b, const char* what) {
  if (a != 0 && b > std::numeric_limits<uint64_t>::max() / a) throw std::overflow_error(std::string(what) + ": size overflow");
  return a * b;
}
static inline uint64_t add_checked(uint64_t a, uint64_t b, const char* what) {
  if (b > std::numeric_limits<uint64_t>::max() - a) throw std::overflow_error(std::string(what) + ": offset overflow");
  return a + b;
}

// ------------------------------------------------------------------ idx-ubyte
// magic = 0x00 0x00 <type 0x08 = u8> <ndim>, then ndim big-endian u32 sizes, then the data.
struct IdxHeader {
  int ndim = 0;
  std::vector<uint64_t> shape;
  uint64_t data_offset = 0, row_bytes = 1;
};

// `hdr` holds the first min(file_size, 20) bytes.  The data of shape[0] rows must fit the file.
static inline IdxHeader parse_idx_header(const uint8_t* hdr, size_t n, uint64_t file_size) {
  if (n < 4) throw std::runtime_error("idx: truncated header");
  if (hdr[0] != 0 || hdr[1] != 0) throw std::runtime_error("idx: bad magic");
  if (hdr[2] != 0x08) throw std::runtime_error("idx: only unsigned-byte idx files are supported");
  IdxHeader h;
  h.ndim = hdr[3];
  if (h.ndim < 1 || h.ndim > 4) throw std::runtime_error("idx: bad rank");
  if (n < size_t(4 + 4 * h.ndim)) throw std::runtime_error("idx: truncated header");
  h.data_offset = 4 + 4 * uint64_t(h.ndim);
  for (int i = 0; i < h.ndim; ++i) {
    h.shape.push_back(be32(hdr + 4 + 4 * i));
    if (i) h.row_bytes = mul_checked(h.row_bytes, h.shape.back(), "idx");
  }
  const uint64_t data = mul_checked(h.row_bytes, h.shape[0], "idx");
  if (add_checked(h.data_offset, data, "idx") > file_size) throw std::runtime_error("idx: file shorter than its header says");
  return h;
}

// ------------------------------------------------------------------ netCDF classic (CDF-1/2/5)
enum NcType : int32_t { NC_BYTE = 1, NC_CHAR = 2, NC_SHORT = 3, NC_INT = 4, NC_FLOAT = 5, NC_DOUBLE = 6,
                        NC_UBYTE = 7, NC_USHORT = 8, NC_UINT = 9, NC_INT64 = 10, NC_UINT64 = 11 };
static const uint32_t TAG_DIM = 0x0A, TAG_VAR = 0x0B, TAG_ATT = 0x0C;

static inline size_t type_size(int32_t t) {
  switch (t) {
    case NC_BYTE: case NC_CHAR: case NC_UBYTE: return 1;
    case NC_SHORT: case NC_USHORT: return 2;
    case NC_INT: case NC_FLOAT: case NC_UINT: return 4;
    case NC_DOUBLE: case NC_INT64: case NC_UINT64: return 8;
  }
  throw std::runtime_error("unknown netCDF type " + std::to_string(t));
}

struct NcDim { std::string name; uint64_t len; };
struct NcAtt { std::string name; int32_t type; uint64_t nelems; std::vector<uint8_t> raw; };
struct NcVar {
  std::string name; std::vector<uint64_t> dimids; std::vector<NcAtt> atts;
  int32_t type; uint64_t vsize; uint64_t begin;
};

// Thrown when the header continues past the bytes given (the reader retries with a larger window).
struct NcTruncated : std::out_of_range {
  NcTruncated() : std::out_of_range("netCDF header truncated") {}
};

class Cursor {
 public:
  Cursor(const uint8_t* b, size_t n, int ver) : b_(b), n_(n), ver_(ver) {}
  uint32_t u32() { need(4); uint32_t v = be32(b_ + p_); p_ += 4; return v; }
  uint64_t u64() { need(8); uint64_t v = be64(b_ + p_); p_ += 8; return v; }
  uint64_t nonneg() { return ver_ == 5 ? u64() : u32(); }
  uint64_t offset() { return ver_ == 1 ? u32() : u64(); }
  std::string name() {
    const uint64_t n = nonneg();
    need(padded(n));
    std::string s(reinterpret_cast<const char*>(b_ + p_), size_t(n));
    p_ += size_t(padded(n));
    return s;
  }
  std::vector<uint8_t> bytes(uint64_t n) {
    need(padded(n));
    std::vector<uint8_t> v(b_ + p_, b_ + p_ + size_t(n));
    p_ += size_t(padded(n));
    return v;
  }
  size_t pos() const { return p_; }

 private:
  static uint64_t padded(uint64_t n) {
    if (n > std::numeric_limits<uint64_t>::max() - 3) throw std::overflow_error("netCDF: length overflow");
    return (n + 3) & ~uint64_t(3);
  }
  void need(uint64_t n) const {
    if (n > n_ - p_) throw NcTruncated();  // p_ <= n_ always: no wrap-around
  }
  const uint8_t* b_;
  size_t n_;
  int ver_;
  size_t p_ = 4;
};

struct NcHeader {
  int ver = 0;
  uint64_t numrecs = 0;
  std::vector<NcDim> dims;
  std::vector<NcAtt> gatts;
  std::vector<NcVar> vars;

  static std::vector<NcAtt> read_atts(Cursor& c) {
    std::vector<NcAtt> out;
    const uint32_t tag = c.u32();
    const uint64_t n = c.nonneg();
    if (tag == 0 && n == 0) return out;
    if (tag != TAG_ATT) throw std::runtime_error("netCDF: bad attribute list tag");
    for (uint64_t i = 0; i < n; ++i) {
      NcAtt a;
      a.name = c.name();
      a.type = int32_t(c.u32());
      a.nelems = c.nonneg();
      a.raw = c.bytes(mul_checked(a.nelems, type_size(a.type), "netCDF attribute"));
      out.push_back(std::move(a));
    }
    return out;
  }

  // Parse the header in b[0, n).  Throws NcTruncated if it continues past n, std::runtime_error /
  // std::overflow_error if it is malformed.  Variables are validated against `file_size`: every
  // dimid exists, the data range begin + product(shape) * type_size does not overflow and lies
  // inside the file (non-record variables).
  void parse(const uint8_t* b, size_t n, uint64_t file_size) {
    if (n < 4 || b[0] != 'C' || b[1] != 'D' || b[2] != 'F') {
      if (n < 4) throw NcTruncated();
      throw std::runtime_error("not a classic netCDF file");
    }
    ver = b[3];
    if (ver != 1 && ver != 2 && ver != 5) throw std::runtime_error("unsupported CDF version");
    Cursor c(b, n, ver);
    dims.clear(); gatts.clear(); vars.clear();
    numrecs = c.nonneg();
    uint32_t tag = c.u32();
    uint64_t cnt = c.nonneg();
    if (!(tag == 0 && cnt == 0)) {
      if (tag != TAG_DIM) throw std::runtime_error("netCDF: bad dim list tag");
      for (uint64_t i = 0; i < cnt; ++i) {
        NcDim d; d.name = c.name(); d.len = c.nonneg();
        dims.push_back(d);
      }
    }
    gatts = read_atts(c);
    tag = c.u32();
    cnt = c.nonneg();
    if (!(tag == 0 && cnt == 0)) {
      if (tag != TAG_VAR) throw std::runtime_error("netCDF: bad var list tag");
      for (uint64_t i = 0; i < cnt; ++i) {
        NcVar v;
        v.name = c.name();
        const uint64_t nd = c.nonneg();
        for (uint64_t k = 0; k < nd; ++k) v.dimids.push_back(c.nonneg());
        v.atts = read_atts(c);
        v.type = int32_t(c.u32());
        v.vsize = c.nonneg();
        v.begin = c.offset();
        uint64_t bytes = type_size(v.type);
        bool record = false;
        for (size_t k = 0; k < v.dimids.size(); ++k) {
          const uint64_t id = v.dimids[k];
          if (id >= dims.size()) throw std::runtime_error("netCDF: dimid out of range");
          if (dims[size_t(id)].len == 0 && k == 0) record = true;  // unlimited (record) dimension
          else bytes = mul_checked(bytes, dims[size_t(id)].len, "netCDF variable");
        }
        if (!record && add_checked(v.begin, bytes, "netCDF variable") > file_size)
          throw std::runtime_error("netCDF: variable " + v.name + " extends past the end of the file");
        vars.push_back(std::move(v));
      }
    }
  }
};

}  // namespace mnist_io
