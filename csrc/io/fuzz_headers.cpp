// Standalone sanitizer/fuzz driver of the header parsers in formats.h (no Python, no pybind11).
//
//   fuzz_headers <seed-file>... [--mutations N] [--seed S]
//
// Every seed file is parsed as an idx-ubyte header and as a netCDF classic header (exactly the
// calls the _io extension makes, with the real file size), then N deterministic mutations of it
// (byte flips, truncations, 0xFF runs = huge lengths, length-field swaps) are parsed from memory.
// Parse errors are expected and counted; the run fails only on a sanitizer report (built with
// -fsanitize=address,undefined -fno-sanitize-recover=all by tests/test_io_fuzz.py), a crash, or an
// exception type the readers do not handle.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <random>
#include <string>
#include <vector>

#include "formats.h"

using namespace mnist_io;

namespace {
struct Tally { long ok = 0, rejected = 0; };

void parse_both(const std::vector<uint8_t>& b, uint64_t file_size, Tally& t) {
  try {
    IdxHeader h = parse_idx_header(b.data(), std::min<size_t>(b.size(), 20), file_size);
    (void)h;
    ++t.ok;
  } catch (const std::runtime_error&) { ++t.rejected; }
  // netCDF: the reader's growing-window loop (4 KiB, x4 ...) over the in-memory "file"
  for (uint64_t win = 64;; win *= 4) {
    const size_t n = size_t(std::min<uint64_t>(win, b.size()));
    NcHeader h;
    try {
      h.parse(b.data(), n, file_size);
      ++t.ok;
      break;
    } catch (const NcTruncated&) {
      if (n == b.size()) { ++t.rejected; break; }
    } catch (const std::runtime_error&) { ++t.rejected; break; }
  }
}
}  // namespace

int main(int argc, char** argv) {
  std::vector<std::string> files;
  long mutations = 2000;
  unsigned seed = 1234;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--mutations") && i + 1 < argc) mutations = std::atol(argv[++i]);
    else if (!std::strcmp(argv[i], "--seed") && i + 1 < argc) seed = unsigned(std::atol(argv[++i]));
    else files.push_back(argv[i]);
  }
  Tally t;
  std::mt19937 rng(seed);
  for (const std::string& f : files) {
    std::ifstream in(f, std::ios::binary);
    std::vector<uint8_t> b((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    parse_both(b, b.size(), t);
    const size_t head = std::min<size_t>(b.size(), 512);  // mutate the header region
    for (long m = 0; m < mutations && head > 0; ++m) {
      std::vector<uint8_t> x(b.begin(), b.begin() + long(std::min<size_t>(b.size(), 4096)));
      const int kind = int(rng() % 5);
      const size_t at = rng() % head;
      if (kind == 0) x[at] ^= uint8_t(1u << (rng() % 8));
      else if (kind == 1) x.resize(at);                               // truncation
      else if (kind == 2) for (size_t k = at; k < std::min(x.size(), at + 8); ++k) x[k] = 0xFF;  // huge length
      else if (kind == 3) for (size_t k = at; k < std::min(x.size(), at + 8); ++k) x[k] = uint8_t(rng());
      else if (x.size() > 16) std::swap(x[at % x.size()], x[rng() % x.size()]);
      const uint64_t fsize = (rng() % 3 == 0) ? uint64_t(rng()) : uint64_t(x.size());  // lie about the size too
      parse_both(x, fsize, t);
    }
  }
  std::printf("fuzz_headers: %ld parsed, %ld rejected\n", t.ok, t.rejected);
  return 0;
}
