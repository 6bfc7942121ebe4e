// ptdump.h — tiny tagged-array container ("PTDUMP01") used to exchange flattened
// scenes, ray batches and HDR images between the host library, the oracle
// harness and the Python tests.  Layout: 8-byte magic, then records of
//   char name[24] | char dtype[8] ("f8","f4","i4","i8","u4") | int64 count | payload
// terminated by a record named "END".  Little-endian, no padding.
#pragma once
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace ptdump {

struct Writer {
  FILE* f = nullptr;
  explicit Writer(const char* path) {
    f = std::fopen(path, "wb");
    if (f) std::fwrite("PTDUMP01", 1, 8, f);
  }
  ~Writer() { close(); }
  bool ok() const { return f != nullptr; }
  void raw(const char* name, const char* dtype, const void* data, int64_t count,
           size_t elem) {
    if (!f) return;
    char nm[24] = {0}, dt[8] = {0};
    std::strncpy(nm, name, 23);
    std::strncpy(dt, dtype, 7);
    std::fwrite(nm, 1, 24, f);
    std::fwrite(dt, 1, 8, f);
    std::fwrite(&count, 8, 1, f);
    if (count > 0) std::fwrite(data, elem, (size_t)count, f);
  }
  void f8(const char* n, const std::vector<double>& v) { raw(n, "f8", v.data(), (int64_t)v.size(), 8); }
  void f4(const char* n, const std::vector<float>& v) { raw(n, "f4", v.data(), (int64_t)v.size(), 4); }
  void i4(const char* n, const std::vector<int32_t>& v) { raw(n, "i4", v.data(), (int64_t)v.size(), 4); }
  void i8(const char* n, const std::vector<int64_t>& v) { raw(n, "i8", v.data(), (int64_t)v.size(), 8); }
  void close() {
    if (!f) return;
    raw("END", "i4", nullptr, 0, 4);
    std::fclose(f);
    f = nullptr;
  }
};

struct Record {
  std::string name, dtype;
  std::vector<char> bytes;
  int64_t count = 0;
};

inline bool read_all(const char* path, std::vector<Record>& out) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return false;
  char magic[8];
  if (std::fread(magic, 1, 8, f) != 8 || std::memcmp(magic, "PTDUMP01", 8) != 0) {
    std::fclose(f);
    return false;
  }
  for (;;) {
    char nm[24], dt[8];
    int64_t count;
    if (std::fread(nm, 1, 24, f) != 24 || std::fread(dt, 1, 8, f) != 8 ||
        std::fread(&count, 8, 1, f) != 1) {
      std::fclose(f);
      return false;
    }
    Record r;
    r.name.assign(nm, strnlen(nm, 24));
    r.dtype.assign(dt, strnlen(dt, 8));
    r.count = count;
    if (r.name == "END") break;
    size_t elem = (r.dtype == "f8" || r.dtype == "i8") ? 8 : 4;
    r.bytes.resize((size_t)count * elem);
    if (count > 0 && std::fread(r.bytes.data(), elem, (size_t)count, f) != (size_t)count) {
      std::fclose(f);
      return false;
    }
    out.push_back(std::move(r));
  }
  std::fclose(f);
  return true;
}

template <class T>
inline bool get(const std::vector<Record>& recs, const char* name, std::vector<T>& v) {
  for (const Record& r : recs) {
    if (r.name == name) {
      v.resize(r.bytes.size() / sizeof(T));
      if (!v.empty()) std::memcpy(v.data(), r.bytes.data(), r.bytes.size());
      return true;
    }
  }
  return false;
}

}  // namespace ptdump
