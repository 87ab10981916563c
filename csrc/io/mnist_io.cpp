// Native MNIST storage formats: idx-ubyte and classic netCDF (CDF-1 / CDF-2 / CDF-5).
//
// Replaces two inherited native stacks of the reference:
//   * torchvision's MNIST idx decode (ddp_tutorial_cpu.py:17-22; the notebook's
//     MnistDataloader.read_images_labels, mnist_to_netcdf.ipynb cell 2 lines 24-45), and
//   * pncpy -> libpnetcdf -> MPI-IO (ROMIO) used by MNISTNetCDF (mnist_pnetcdf_cpu_mp.py:18-49)
//     and by the converter's to_nc() (notebook cell 2 lines 83-104).
// There is no MPI here: a reader opens the file, parses the header once, and pulls
// hyperslabs with pread() from a small thread pool straight into caller memory
// (typically a pinned host tensor that is then hipMemcpyAsync'ed into HBM).
//
// Format (netCDF classic spec, CDF-5 = "64BIT_DATA"): magic "CDF"+ver; numrecs;
// dim_list; gatt_list; var_list.  Big-endian.  CDF-5 widens NON_NEG / dimids /
// vsize / begin to 64 bit; CDF-2 widens only begin.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace mnist_io {

// ------------------------------------------------------------------ big-endian helpers
static inline uint32_t be32(const uint8_t* p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | uint32_t(p[3]);
}
static inline uint64_t be64(const uint8_t* p) { return (uint64_t(be32(p)) << 32) | be32(p + 4); }
static inline void put32(std::vector<uint8_t>& o, uint32_t v) {
  for (int s = 24; s >= 0; s -= 8) o.push_back(uint8_t(v >> s));
}
static inline void put64(std::vector<uint8_t>& o, uint64_t v) {
  put32(o, uint32_t(v >> 32));
  put32(o, uint32_t(v));
}

struct Fd {
  int fd = -1;
  explicit Fd(int f) : fd(f) {}
  ~Fd() { if (fd >= 0) ::close(fd); }
  Fd(const Fd&) = delete;
  Fd& operator=(const Fd&) = delete;
};

static void pread_all(int fd, void* dst, size_t n, uint64_t off) {
  uint8_t* d = static_cast<uint8_t*>(dst);
  while (n) {
    ssize_t r = ::pread(fd, d, n, static_cast<off_t>(off));
    if (r < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error(std::string("pread failed: ") + std::strerror(errno));
    }
    if (r == 0) throw std::runtime_error("unexpected end of file");
    d += r; n -= size_t(r); off += uint64_t(r);
  }
}

static void write_all(int fd, const void* src, size_t n) {
  const uint8_t* s = static_cast<const uint8_t*>(src);
  while (n) {
    ssize_t r = ::write(fd, s, n);
    if (r < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error(std::string("write failed: ") + std::strerror(errno));
    }
    s += r; n -= size_t(r);
  }
}

// Parallel pread of [off, off+n) into dst using up to `threads` workers (large reads only).
static void pread_parallel(int fd, uint8_t* dst, size_t n, uint64_t off, int threads) {
  const size_t chunk = size_t(4) << 20;
  if (threads <= 1 || n <= chunk) { pread_all(fd, dst, n, off); return; }
  size_t nchunks = (n + chunk - 1) / chunk;
  int nt = int(std::min<size_t>(size_t(threads), nchunks));
  std::vector<std::thread> pool;
  std::vector<std::string> errs(nt);
  for (int t = 0; t < nt; ++t) {
    pool.emplace_back([&, t] {
      try {
        for (size_t c = size_t(t); c < nchunks; c += size_t(nt)) {
          size_t b = c * chunk, e = std::min(n, b + chunk);
          pread_all(fd, dst + b, e - b, off + b);
        }
      } catch (const std::exception& ex) { errs[t] = ex.what(); }
    });
  }
  for (auto& th : pool) th.join();
  for (auto& e : errs) if (!e.empty()) throw std::runtime_error(e);
}

// ------------------------------------------------------------------ idx-ubyte
// magic = 0x00 0x00 <type> <ndim>, then ndim big-endian u32 sizes, then data.
// MNIST: labels 2049 (>II), images 2051 (>IIII), type 0x08 = unsigned byte.
py::array_t<uint8_t> idx_read(const std::string& path, int64_t limit) {
  int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) throw std::runtime_error("cannot open " + path + ": " + std::strerror(errno));
  Fd guard(fd);
  uint8_t hdr[4];
  pread_all(fd, hdr, 4, 0);
  if (hdr[0] != 0 || hdr[1] != 0) throw std::runtime_error(path + ": bad idx magic");
  if (hdr[2] != 0x08) throw std::runtime_error(path + ": only unsigned-byte idx files are supported");
  int ndim = hdr[3];
  if (ndim < 1 || ndim > 4) throw std::runtime_error(path + ": bad idx rank");
  std::vector<uint8_t> dimb(4 * size_t(ndim));
  pread_all(fd, dimb.data(), dimb.size(), 4);
  std::vector<ssize_t> shape(ndim);
  size_t per = 1;
  for (int i = 0; i < ndim; ++i) {
    shape[i] = ssize_t(be32(&dimb[4 * i]));
    if (i) per *= size_t(shape[i]);
  }
  if (limit >= 0 && limit < shape[0]) shape[0] = limit;
  py::array_t<uint8_t> out(shape);
  size_t bytes = per * size_t(shape[0]);
  {
    py::gil_scoped_release nogil;
    pread_parallel(fd, out.mutable_data(), bytes, 4 + 4 * uint64_t(ndim), 4);
  }
  return out;
}

void idx_write(const std::string& path, py::array_t<uint8_t, py::array::c_style | py::array::forcecast> a) {
  if (a.ndim() < 1 || a.ndim() > 4) throw std::runtime_error("idx_write: rank must be 1..4");
  std::vector<uint8_t> h = {0, 0, 0x08, uint8_t(a.ndim())};
  for (int i = 0; i < a.ndim(); ++i) put32(h, uint32_t(a.shape(i)));
  int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) throw std::runtime_error("cannot create " + path);
  Fd guard(fd);
  write_all(fd, h.data(), h.size());
  write_all(fd, a.data(), size_t(a.nbytes()));
}

// ------------------------------------------------------------------ netCDF classic
enum NcType : int32_t { NC_BYTE = 1, NC_CHAR = 2, NC_SHORT = 3, NC_INT = 4, NC_FLOAT = 5, NC_DOUBLE = 6,
                        NC_UBYTE = 7, NC_USHORT = 8, NC_UINT = 9, NC_INT64 = 10, NC_UINT64 = 11 };
static const uint32_t TAG_DIM = 0x0A, TAG_VAR = 0x0B, TAG_ATT = 0x0C;

static size_t type_size(int32_t t) {
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

class Cursor {
 public:
  Cursor(const std::vector<uint8_t>& b, int ver) : b_(b), ver_(ver) {}
  uint32_t u32() { need(4); uint32_t v = be32(&b_[p_]); p_ += 4; return v; }
  uint64_t u64() { need(8); uint64_t v = be64(&b_[p_]); p_ += 8; return v; }
  uint64_t nonneg() { return ver_ == 5 ? u64() : u32(); }
  uint64_t offset() { return ver_ == 1 ? u32() : u64(); }
  std::string name() {
    uint64_t n = nonneg();
    need(n);
    std::string s(reinterpret_cast<const char*>(&b_[p_]), size_t(n));
    p_ += (n + 3) & ~uint64_t(3);
    return s;
  }
  std::vector<uint8_t> bytes(uint64_t n) {
    need(n);
    std::vector<uint8_t> v(b_.begin() + p_, b_.begin() + p_ + n);
    p_ += (n + 3) & ~uint64_t(3);
    return v;
  }
  size_t pos() const { return p_; }
  bool has(size_t n) const { return p_ + n <= b_.size(); }

 private:
  void need(uint64_t n) const {
    if (p_ + n > b_.size()) throw std::out_of_range("header truncated");
  }
  const std::vector<uint8_t>& b_;
  int ver_;
  size_t p_ = 4;
};

static std::vector<NcAtt> read_atts(Cursor& c) {
  std::vector<NcAtt> out;
  uint32_t tag = c.u32();
  uint64_t n = c.nonneg();
  if (tag == 0 && n == 0) return out;
  if (tag != TAG_ATT) throw std::runtime_error("bad attribute list tag");
  for (uint64_t i = 0; i < n; ++i) {
    NcAtt a;
    a.name = c.name();
    a.type = int32_t(c.u32());
    a.nelems = c.nonneg();
    a.raw = c.bytes(a.nelems * type_size(a.type));
    out.push_back(std::move(a));
  }
  return out;
}

class NcFile {
 public:
  explicit NcFile(const std::string& path) : path_(path) {
    fd_ = ::open(path.c_str(), O_RDONLY);
    if (fd_ < 0) throw std::runtime_error("cannot open " + path + ": " + std::strerror(errno));
    struct stat st;
    ::fstat(fd_, &st);
    file_size_ = uint64_t(st.st_size);
    // Headers of MNIST-sized files are a few hundred bytes; grow the window if needed.
    for (size_t win = 4096;; win *= 4) {
      size_t n = size_t(std::min<uint64_t>(win, file_size_));
      std::vector<uint8_t> buf(n);
      pread_all(fd_, buf.data(), n, 0);
      try {
        parse(buf);
        break;
      } catch (const std::out_of_range&) {
        if (n == file_size_) throw std::runtime_error(path + ": truncated netCDF header");
      }
    }
  }
  ~NcFile() { if (fd_ >= 0) ::close(fd_); }

  int version() const { return ver_; }
  const std::string& path() const { return path_; }
  std::vector<std::pair<std::string, uint64_t>> dims() const {
    std::vector<std::pair<std::string, uint64_t>> o;
    for (auto& d : dims_) o.emplace_back(d.name, d.len);
    return o;
  }
  std::vector<std::string> variables() const {
    std::vector<std::string> o;
    for (auto& v : vars_) o.push_back(v.name);
    return o;
  }
  const NcVar& var(const std::string& n) const {
    for (auto& v : vars_) if (v.name == n) return v;
    throw std::runtime_error(path_ + ": no variable " + n);
  }
  std::vector<uint64_t> shape(const std::string& n) const {
    std::vector<uint64_t> s;
    for (auto id : var(n).dimids) s.push_back(dims_.at(size_t(id)).len);
    return s;
  }
  int32_t vtype(const std::string& n) const { return var(n).type; }
  uint64_t begin(const std::string& n) const { return var(n).begin; }
  py::dict var_info(const std::string& n) const {
    const NcVar& v = var(n);
    py::dict d;
    d["type"] = v.type; d["vsize"] = v.vsize; d["begin"] = v.begin;
    d["shape"] = shape(n);
    std::vector<std::string> dn;
    for (auto id : v.dimids) dn.push_back(dims_.at(size_t(id)).name);
    d["dims"] = dn;
    return d;
  }
  py::dict global_attributes() const {
    py::dict d;
    for (auto& a : gatts_) d[py::str(a.name)] = py::bytes(reinterpret_cast<const char*>(a.raw.data()), a.raw.size());
    return d;
  }

  // rows [start, start+count) of a non-record variable (row = slice along dim 0).
  py::array read_rows(const std::string& n, uint64_t start, int64_t count, int threads) const {
    const NcVar& v = var(n);
    auto shp = shape(n);
    if (shp.empty()) throw std::runtime_error("scalar variable");
    uint64_t nrows = shp[0];
    uint64_t cnt = count < 0 ? nrows - std::min(start, nrows) : uint64_t(count);
    if (start + cnt > nrows) throw std::out_of_range("read_rows: rows out of range");
    uint64_t row_bytes = type_size(v.type);
    for (size_t i = 1; i < shp.size(); ++i) row_bytes *= shp[i];
    std::vector<ssize_t> oshape = {ssize_t(cnt)};
    for (size_t i = 1; i < shp.size(); ++i) oshape.push_back(ssize_t(shp[i]));
    py::array out(dtype_of(v.type), oshape);
    uint8_t* dst = static_cast<uint8_t*>(out.mutable_data());
    size_t bytes = size_t(cnt * row_bytes);
    {
      py::gil_scoped_release nogil;
      pread_parallel(fd_, dst, bytes, v.begin + start * row_bytes, threads);
      fix_endian(dst, bytes, type_size(v.type));
    }
    return out;
  }

  // Same, but into caller memory (e.g. a pinned host tensor): returns bytes written.
  uint64_t read_rows_into(const std::string& n, uint64_t start, uint64_t count, uintptr_t dst_ptr,
                          uint64_t dst_bytes, int threads) const {
    const NcVar& v = var(n);
    auto shp = shape(n);
    uint64_t row_bytes = type_size(v.type);
    for (size_t i = 1; i < shp.size(); ++i) row_bytes *= shp[i];
    if (start + count > shp[0]) throw std::out_of_range("read_rows_into: rows out of range");
    uint64_t bytes = count * row_bytes;
    if (bytes > dst_bytes) throw std::runtime_error("read_rows_into: destination too small");
    py::gil_scoped_release nogil;
    uint8_t* dst = reinterpret_cast<uint8_t*>(dst_ptr);
    pread_parallel(fd_, dst, size_t(bytes), v.begin + start * row_bytes, threads);
    fix_endian(dst, size_t(bytes), type_size(v.type));
    return bytes;
  }

  // One element (the reference's per-sample independent get_var, mnist_pnetcdf_cpu_mp.py:43-46).
  py::array read_row(const std::string& n, uint64_t index) const { return read_rows(n, index, 1, 1); }

 private:
  static py::dtype dtype_of(int32_t t) {
    switch (t) {
      case NC_BYTE: return py::dtype("i1");
      case NC_CHAR: case NC_UBYTE: return py::dtype("u1");
      case NC_SHORT: return py::dtype("<i2");
      case NC_USHORT: return py::dtype("<u2");
      case NC_INT: return py::dtype("<i4");
      case NC_UINT: return py::dtype("<u4");
      case NC_FLOAT: return py::dtype("<f4");
      case NC_DOUBLE: return py::dtype("<f8");
      case NC_INT64: return py::dtype("<i8");
      case NC_UINT64: return py::dtype("<u8");
    }
    throw std::runtime_error("unknown type");
  }
  static void fix_endian(uint8_t* p, size_t bytes, size_t w) {
    if (w == 1) return;
    for (size_t i = 0; i + w <= bytes; i += w) std::reverse(p + i, p + i + w);
  }
  void parse(const std::vector<uint8_t>& b) {
    if (b.size() < 4 || b[0] != 'C' || b[1] != 'D' || b[2] != 'F')
      throw std::runtime_error(path_ + ": not a classic netCDF file");
    ver_ = b[3];
    if (ver_ != 1 && ver_ != 2 && ver_ != 5) throw std::runtime_error(path_ + ": unsupported CDF version");
    Cursor c(b, ver_);
    dims_.clear(); gatts_.clear(); vars_.clear();
    numrecs_ = c.nonneg();
    uint32_t tag = c.u32();
    uint64_t n = c.nonneg();
    if (!(tag == 0 && n == 0)) {
      if (tag != TAG_DIM) throw std::runtime_error("bad dim list tag");
      for (uint64_t i = 0; i < n; ++i) {
        NcDim d; d.name = c.name(); d.len = c.nonneg();
        dims_.push_back(d);
      }
    }
    gatts_ = read_atts(c);
    tag = c.u32();
    n = c.nonneg();
    if (!(tag == 0 && n == 0)) {
      if (tag != TAG_VAR) throw std::runtime_error("bad var list tag");
      for (uint64_t i = 0; i < n; ++i) {
        NcVar v;
        v.name = c.name();
        uint64_t nd = c.nonneg();
        for (uint64_t k = 0; k < nd; ++k) v.dimids.push_back(c.nonneg());
        v.atts = read_atts(c);
        v.type = int32_t(c.u32());
        v.vsize = c.nonneg();
        v.begin = c.offset();
        for (auto id : v.dimids)
          if (id >= dims_.size()) throw std::runtime_error("dimid out of range");
        vars_.push_back(std::move(v));
      }
    }
  }
  std::string path_;
  int fd_ = -1;
  int ver_ = 0;
  uint64_t file_size_ = 0, numrecs_ = 0;
  std::vector<NcDim> dims_;
  std::vector<NcAtt> gatts_;
  std::vector<NcVar> vars_;
};

// CDF-5 writer for non-record variables.  Semantics of the notebook's to_nc()
// (dims Y, X, idx; vars images(idx,Y,X), labels(idx), NC_UBYTE), but written
// once by one process with one bulk write per variable (survey quirk Q17),
// data section aligned like PnetCDF's default (512 B).
void cdf5_write(const std::string& path,
                const std::vector<std::pair<std::string, uint64_t>>& dims,
                const std::vector<std::tuple<std::string, std::vector<int>, py::array>>& vars,
                uint64_t align) {
  std::vector<uint8_t> h = {'C', 'D', 'F', 5};
  put64(h, 0);  // numrecs
  auto put_name = [&](const std::string& s) {
    put64(h, s.size());
    h.insert(h.end(), s.begin(), s.end());
    while (h.size() % 4) h.push_back(0);
  };
  if (dims.empty()) { put32(h, 0); put64(h, 0); }
  else {
    put32(h, TAG_DIM); put64(h, dims.size());
    for (auto& d : dims) { put_name(d.first); put64(h, d.second); }
  }
  put32(h, 0); put64(h, 0);  // no global attributes
  struct Pending { size_t begin_pos; uint64_t vsize; const py::array* arr; };
  std::vector<Pending> pend;
  if (vars.empty()) { put32(h, 0); put64(h, 0); }
  else {
    put32(h, TAG_VAR); put64(h, vars.size());
    for (auto& v : vars) {
      const std::string& name = std::get<0>(v);
      const std::vector<int>& dimids = std::get<1>(v);
      const py::array& arr = std::get<2>(v);
      int32_t t;
      char kind = arr.dtype().kind();
      size_t isz = size_t(arr.itemsize());
      if (kind == 'u' && isz == 1) t = NC_UBYTE;
      else if (kind == 'i' && isz == 1) t = NC_BYTE;
      else if (kind == 'i' && isz == 2) t = NC_SHORT;
      else if (kind == 'u' && isz == 2) t = NC_USHORT;
      else if (kind == 'i' && isz == 4) t = NC_INT;
      else if (kind == 'u' && isz == 4) t = NC_UINT;
      else if (kind == 'f' && isz == 4) t = NC_FLOAT;
      else if (kind == 'f' && isz == 8) t = NC_DOUBLE;
      else if (kind == 'i' && isz == 8) t = NC_INT64;
      else if (kind == 'u' && isz == 8) t = NC_UINT64;
      else throw std::runtime_error("cdf5_write: unsupported dtype for " + name);
      uint64_t nel = 1;
      for (int id : dimids) {
        if (id < 0 || size_t(id) >= dims.size()) throw std::runtime_error("cdf5_write: bad dimid");
        nel *= dims[size_t(id)].second;
      }
      if (nel != uint64_t(arr.size())) throw std::runtime_error("cdf5_write: shape mismatch for " + name);
      put_name(name);
      put64(h, dimids.size());
      for (int id : dimids) put64(h, uint64_t(id));
      put32(h, 0); put64(h, 0);  // no variable attributes
      put32(h, uint32_t(t));
      uint64_t vsize = (nel * isz + 3) & ~uint64_t(3);
      put64(h, vsize);
      pend.push_back({h.size(), vsize, &arr});
      put64(h, 0);  // begin, patched below
    }
  }
  if (align == 0) align = 4;
  uint64_t off = (h.size() + align - 1) / align * align;
  for (auto& p : pend) {
    uint64_t b = off;
    for (int s = 0; s < 8; ++s) h[p.begin_pos + size_t(s)] = uint8_t(b >> (56 - 8 * s));
    off = b + (p.vsize + align - 1) / align * align;
  }
  int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) throw std::runtime_error("cannot create " + path);
  Fd guard(fd);
  write_all(fd, h.data(), h.size());
  uint64_t cur = h.size();
  std::vector<uint8_t> zeros(size_t(align), 0);
  for (size_t i = 0; i < pend.size(); ++i) {
    uint64_t b = 0;
    for (int s = 0; s < 8; ++s) b = (b << 8) | h[pend[i].begin_pos + size_t(s)];
    while (cur < b) { size_t z = size_t(std::min<uint64_t>(b - cur, zeros.size())); write_all(fd, zeros.data(), z); cur += z; }
    const py::array& arr = *pend[i].arr;
    py::array c = py::array::ensure(arr, py::array::c_style);
    size_t isz = size_t(c.itemsize()), nb = size_t(c.nbytes());
    if (isz == 1) write_all(fd, c.data(), nb);
    else {  // to big-endian
      std::vector<uint8_t> tmp(static_cast<const uint8_t*>(c.data()), static_cast<const uint8_t*>(c.data()) + nb);
      for (size_t k = 0; k + isz <= nb; k += isz) std::reverse(tmp.begin() + long(k), tmp.begin() + long(k + isz));
      write_all(fd, tmp.data(), nb);
    }
    cur += nb;
    while (cur < b + pend[i].vsize) { write_all(fd, zeros.data(), 1); cur += 1; }
  }
}

}  // namespace mnist_io

PYBIND11_MODULE(_io, m) {
  using namespace mnist_io;
  m.doc() = "native idx-ubyte and CDF-1/2/5 (PnetCDF classic) readers/writers";
  m.def("idx_read", &idx_read, py::arg("path"), py::arg("limit") = -1);
  m.def("idx_write", &idx_write, py::arg("path"), py::arg("array"));
  m.def("cdf5_write", &cdf5_write, py::arg("path"), py::arg("dims"), py::arg("vars"), py::arg("align") = 512);
  py::class_<NcFile>(m, "NcFile")
      .def(py::init<const std::string&>())
      .def_property_readonly("version", &NcFile::version)
      .def_property_readonly("path", &NcFile::path)
      .def("dims", &NcFile::dims)
      .def("variables", &NcFile::variables)
      .def("shape", &NcFile::shape)
      .def("begin", &NcFile::begin)
      .def("var_info", &NcFile::var_info)
      .def("global_attributes", &NcFile::global_attributes)
      .def("read_rows", &NcFile::read_rows, py::arg("name"), py::arg("start") = 0, py::arg("count") = -1,
           py::arg("threads") = 4)
      .def("read_rows_into", &NcFile::read_rows_into, py::arg("name"), py::arg("start"), py::arg("count"),
           py::arg("dst_ptr"), py::arg("dst_bytes"), py::arg("threads") = 4)
      .def("read_row", &NcFile::read_row);
}
