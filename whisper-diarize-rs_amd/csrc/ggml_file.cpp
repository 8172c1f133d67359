#include "ggml_file.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <stdexcept>

namespace wdr {

namespace {

[[noreturn]] void bad(const std::string& why) { throw std::runtime_error("failed to open model: " + why); }

// IEEE binary16 <-> binary32 (round to nearest even), host side
float h2f(uint16_t h) {
  const uint32_t s = (uint32_t)(h & 0x8000) << 16;
  uint32_t e = (h >> 10) & 0x1f, m = h & 0x3ff, u;
  if (e == 0) {
    if (m == 0) {
      u = s;
    } else {   // subnormal
      e = 127 - 15 + 1;
      while (!(m & 0x400)) {
        m <<= 1;
        --e;
      }
      m &= 0x3ff;
      u = s | (e << 23) | (m << 13);
    }
  } else if (e == 31) {
    u = s | 0x7f800000 | (m << 13);
  } else {
    u = s | ((e + 127 - 15) << 23) | (m << 13);
  }
  float f;
  memcpy(&f, &u, 4);
  return f;
}

uint16_t f2h(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  const uint32_t s = (u >> 16) & 0x8000;
  const int32_t e = (int32_t)((u >> 23) & 0xff) - 127 + 15;
  uint32_t m = u & 0x7fffff;
  if (((u >> 23) & 0xff) == 0xff) return (uint16_t)(s | 0x7c00 | (m ? 0x200 : 0));   // inf / nan
  if (e >= 31) return (uint16_t)(s | 0x7c00);
  if (e <= 0) {
    if (e < -10) return (uint16_t)s;
    m |= 0x800000;
    const int shift = 14 - e;
    uint32_t r = m >> shift;
    const uint32_t rem = m & ((1u << shift) - 1), half = 1u << (shift - 1);
    if (rem > half || (rem == half && (r & 1))) ++r;
    return (uint16_t)(s | r);
  }
  uint32_t r = ((uint32_t)e << 10) | (m >> 13);
  const uint32_t rem = m & 0x1fff;
  if (rem > 0x1000 || (rem == 0x1000 && (r & 1))) ++r;
  return (uint16_t)(s | r);
}

struct Reader {
  const char* p;
  const char* end;
  template <typename T>
  T get() {
    if ((size_t)(end - p) < sizeof(T)) bad("truncated file");
    T v;
    memcpy(&v, p, sizeof(T));
    p += sizeof(T);
    return v;
  }
  const char* take(size_t n) {
    if ((size_t)(end - p) < n) bad("truncated file");
    const char* q = p;
    p += n;
    return q;
  }
};

}  // namespace

GgmlFile::GgmlFile(const std::string& path) {
  const int fd = open(path.c_str(), O_RDONLY);
  if (fd < 0) bad("cannot open " + path);
  struct stat st;
  if (fstat(fd, &st) != 0 || st.st_size < 64) {
    close(fd);
    bad("not a ggml model file: " + path);
  }
  size_ = (size_t)st.st_size;
  map_ = mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd, 0);
  close(fd);
  if (map_ == MAP_FAILED) {
    map_ = nullptr;
    bad("cannot map " + path);
  }
  Reader r{(const char*)map_, (const char*)map_ + size_};
  if (r.get<uint32_t>() != 0x67676d6cu) bad("bad magic (not a whisper.cpp ggml file): " + path);
  for (int i = 0; i < 11; ++i) hp[i] = r.get<int32_t>();
  n_mel = r.get<int32_t>();
  n_fft = r.get<int32_t>();
  if (n_mel <= 0 || n_fft <= 0 || n_mel > 512 || n_fft > 4096) bad("bad mel filter header");
  filters.resize((size_t)n_mel * n_fft);
  memcpy(filters.data(), r.take(filters.size() * 4), filters.size() * 4);
  const int32_t nv = r.get<int32_t>();
  if (nv < 0 || nv > 1000000) bad("bad vocabulary size");
  vocab.resize(nv);
  for (int i = 0; i < nv; ++i) {
    const uint32_t len = r.get<uint32_t>();
    if (len > 4096) bad("bad token length");
    vocab[i].assign(r.take(len), len);
  }
  while (r.p < r.end) {
    const int32_t nd = r.get<int32_t>(), nl = r.get<int32_t>(), type = r.get<int32_t>();
    if (nd < 1 || nd > 4 || nl <= 0 || nl > 1024) bad("bad tensor header");
    if (type != 0 && type != 1) bad("unsupported tensor type " + std::to_string(type) + " (only f32 / f16 models)");
    GgmlTensor t;
    t.type = type;
    for (int i = 0; i < nd; ++i) t.ne.push_back(r.get<int32_t>());
    const std::string name(r.take(nl), nl);
    t.data = r.take((size_t)t.n_elem() * (type == 0 ? 4 : 2));
    tensors[name] = t;
  }
}

GgmlFile::~GgmlFile() {
  if (map_) munmap(map_, size_);
}

const GgmlTensor& GgmlFile::get(const std::string& name) const {
  auto it = tensors.find(name);
  if (it == tensors.end()) bad("tensor '" + name + "' not found");
  return it->second;
}

std::vector<float> GgmlFile::as_f32(const std::string& name, int64_t n) const {
  const GgmlTensor& t = get(name);
  if (t.n_elem() != n) bad("tensor '" + name + "' has " + std::to_string(t.n_elem()) + " elements, expected " +
                           std::to_string(n));
  std::vector<float> out((size_t)n);
  if (t.type == 0) {
    memcpy(out.data(), t.data, (size_t)n * 4);
  } else {
    for (int64_t i = 0; i < n; ++i) {
      uint16_t h;
      memcpy(&h, t.data + 2 * i, 2);
      out[i] = h2f(h);
    }
  }
  return out;
}

std::vector<uint16_t> GgmlFile::as_f16(const std::string& name, int64_t n) const {
  const GgmlTensor& t = get(name);
  if (t.n_elem() != n) bad("tensor '" + name + "' has " + std::to_string(t.n_elem()) + " elements, expected " +
                           std::to_string(n));
  std::vector<uint16_t> out((size_t)n);
  if (t.type == 1) {
    memcpy(out.data(), t.data, (size_t)n * 2);
  } else {
    for (int64_t i = 0; i < n; ++i) {
      float f;
      memcpy(&f, t.data + 4 * i, 4);
      out[i] = f2h(f);
    }
  }
  return out;
}

}  // namespace wdr
