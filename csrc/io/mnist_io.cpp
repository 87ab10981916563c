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

#include "formats.h"

namespace py = pybind11;

namespace mnist_io {

// ------------------------------------------------------------------ big-endian writers
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
  struct stat st;
  if (::fstat(fd, &st) != 0) throw std::runtime_error("cannot stat " + path);
  const uint64_t fsize = uint64_t(st.st_size);
  uint8_t hdr[20] = {0};
  const size_t hn = size_t(std::min<uint64_t>(fsize, sizeof(hdr)));
  pread_all(fd, hdr, hn, 0);
  IdxHeader h;
  try {
    h = parse_idx_header(hdr, hn, fsize);
  } catch (const std::exception& e) {
    throw std::runtime_error(path + ": " + e.what());
  }
  std::vector<ssize_t> shape(h.shape.begin(), h.shape.end());
  if (limit >= 0 && limit < shape[0]) shape[0] = limit;
  py::array_t<uint8_t> out(shape);
  size_t bytes = size_t(h.row_bytes * uint64_t(shape[0]));  // <= file size (checked by the parser)
  {
    py::gil_scoped_release nogil;
    pread_parallel(fd, out.mutable_data(), bytes, h.data_offset, 4);
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

// ------------------------------------------------------------------ netCDF classic (parser: formats.h)
class NcFile {
 public:
  explicit NcFile(const std::string& path) : path_(path) {
    fd_ = ::open(path.c_str(), O_RDONLY);
    if (fd_ < 0) throw std::runtime_error("cannot open " + path + ": " + std::strerror(errno));
    struct stat st;
    if (::fstat(fd_, &st) != 0) { ::close(fd_); throw std::runtime_error("cannot stat " + path); }
    file_size_ = uint64_t(st.st_size);
    // Headers of MNIST-sized files are a few hundred bytes; grow the window if needed.
    try {
      for (uint64_t win = 4096;; win *= 4) {
        const size_t n = size_t(std::min<uint64_t>(win, file_size_));
        std::vector<uint8_t> buf(n);
        pread_all(fd_, buf.data(), n, 0);
        try {
          h_.parse(buf.data(), n, file_size_);
          break;
        } catch (const NcTruncated&) {
          if (n == file_size_) throw std::runtime_error("truncated netCDF header");
        }
      }
    } catch (const std::exception& e) {
      ::close(fd_);
      fd_ = -1;
      throw std::runtime_error(path + ": " + e.what());
    }
  }
  ~NcFile() { if (fd_ >= 0) ::close(fd_); }

  int version() const { return h_.ver; }
  const std::string& path() const { return path_; }
  std::vector<std::pair<std::string, uint64_t>> dims() const {
    std::vector<std::pair<std::string, uint64_t>> o;
    for (auto& d : h_.dims) o.emplace_back(d.name, d.len);
    return o;
  }
  std::vector<std::string> variables() const {
    std::vector<std::string> o;
    for (auto& v : h_.vars) o.push_back(v.name);
    return o;
  }
  const NcVar& var(const std::string& n) const {
    for (auto& v : h_.vars) if (v.name == n) return v;
    throw std::runtime_error(path_ + ": no variable " + n);
  }
  std::vector<uint64_t> shape(const std::string& n) const {
    std::vector<uint64_t> s;
    for (auto id : var(n).dimids) s.push_back(h_.dims.at(size_t(id)).len);
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
    for (auto id : v.dimids) dn.push_back(h_.dims.at(size_t(id)).name);
    d["dims"] = dn;
    return d;
  }
  py::dict global_attributes() const {
    py::dict d;
    for (auto& a : h_.gatts) d[py::str(a.name)] = py::bytes(reinterpret_cast<const char*>(a.raw.data()), a.raw.size());
    return d;
  }

  // rows [start, start+count) of a non-record variable (row = slice along dim 0).
  py::array read_rows(const std::string& n, uint64_t start, int64_t count, int threads) const {
    const NcVar& v = var(n);
    auto shp = shape(n);
    if (shp.empty()) throw std::runtime_error("scalar variable");
    uint64_t nrows = shp[0];
    uint64_t cnt = count < 0 ? nrows - std::min(start, nrows) : uint64_t(count);
    if (start > nrows || cnt > nrows - start) throw std::out_of_range("read_rows: rows out of range");
    const uint64_t row_bytes = row_size(v, shp);
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
    if (shp.empty()) throw std::runtime_error("scalar variable");
    const uint64_t row_bytes = row_size(v, shp);
    if (start > shp[0] || count > shp[0] - start) throw std::out_of_range("read_rows_into: rows out of range");
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
  // bytes of one row (slice along dim 0); the whole variable was checked to fit the file at parse time
  static uint64_t row_size(const NcVar& v, const std::vector<uint64_t>& shp) {
    uint64_t r = type_size(v.type);
    for (size_t i = 1; i < shp.size(); ++i) r = mul_checked(r, shp[i], "netCDF row");
    return r;
  }
  static void fix_endian(uint8_t* p, size_t bytes, size_t w) {
    if (w == 1) return;
    for (size_t i = 0; i + w <= bytes; i += w) std::reverse(p + i, p + i + w);
  }
  std::string path_;
  int fd_ = -1;
  uint64_t file_size_ = 0;
  NcHeader h_;
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
