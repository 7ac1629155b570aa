// safetensors reader/writer (replaces the Rust `safetensors` wheel; reference comfy/utils.py:13-14,
// :32-36, :285-291 and nodes.py:20, :579).
//
// Reader: mmap the file (MAP_PRIVATE so tensor views may be handed out writable without touching
// the file), parse the little-endian u64 header length + JSON header with a small strict parser,
// validate every tensor's byte range against the data section, and expose zero-copy pointers.
// `copy_many` fans page-faulting copies out over threads (a cold multi-GB checkpoint is bounded by
// the page cache / NVMe, not by one memcpy thread).
// Writer: header JSON with sorted-by-insertion tensors, 8-byte aligned data section.
#include "runtime.h"

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <fcntl.h>
#include <stdexcept>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>

namespace cgs {

MappedFile::MappedFile(const std::string& path) {
  int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) throw std::runtime_error("safetensors: cannot open " + path);
  struct stat st;
  if (fstat(fd, &st) != 0) {
    ::close(fd);
    throw std::runtime_error("safetensors: stat failed " + path);
  }
  size_ = size_t(st.st_size);
  if (size_ > 0) {
    void* m = mmap(nullptr, size_, PROT_READ | PROT_WRITE, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) {
      ::close(fd);
      throw std::runtime_error("safetensors: mmap failed " + path);
    }
    base_ = static_cast<uint8_t*>(m);
  }
  ::close(fd);
}

MappedFile::~MappedFile() {
  if (base_) munmap(base_, size_);
}

namespace {

// Minimal JSON reader for the safetensors header: objects, arrays, strings, integers, literals.
struct Json {
  const char* p;
  const char* e;

  [[noreturn]] void fail(const char* what) const {
    throw std::runtime_error(std::string("safetensors header: ") + what);
  }
  void ws() {
    while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }
  bool eat(char c) {
    ws();
    if (p < e && *p == c) { ++p; return true; }
    return false;
  }
  void expect(char c) {
    if (!eat(c)) fail("unexpected character");
  }
  static void put_utf8(std::string& s, uint32_t cp) {
    if (cp < 0x80) s += char(cp);
    else if (cp < 0x800) { s += char(0xC0 | (cp >> 6)); s += char(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) {
      s += char(0xE0 | (cp >> 12)); s += char(0x80 | ((cp >> 6) & 0x3F)); s += char(0x80 | (cp & 0x3F));
    } else {
      s += char(0xF0 | (cp >> 18)); s += char(0x80 | ((cp >> 12) & 0x3F));
      s += char(0x80 | ((cp >> 6) & 0x3F)); s += char(0x80 | (cp & 0x3F));
    }
  }
  uint32_t hex4() {
    if (e - p < 4) fail("short \\u escape");
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i, ++p) {
      char c = *p;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= uint32_t(c - '0');
      else if (c >= 'a' && c <= 'f') v |= uint32_t(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= uint32_t(c - 'A' + 10);
      else fail("bad \\u escape");
    }
    return v;
  }
  std::string str() {
    ws();
    if (p >= e || *p != '"') fail("expected string");
    ++p;
    std::string s;
    while (p < e && *p != '"') {
      char c = *p++;
      if (c != '\\') { s += c; continue; }
      if (p >= e) fail("bad escape");
      char x = *p++;
      switch (x) {
        case '"': s += '"'; break;
        case '\\': s += '\\'; break;
        case '/': s += '/'; break;
        case 'b': s += '\b'; break;
        case 'f': s += '\f'; break;
        case 'n': s += '\n'; break;
        case 'r': s += '\r'; break;
        case 't': s += '\t'; break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
            p += 2;
            uint32_t lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(s, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    if (p >= e) fail("unterminated string");
    ++p;
    return s;
  }
  int64_t integer() {
    ws();
    bool neg = false;
    if (p < e && *p == '-') { neg = true; ++p; }
    if (p >= e || *p < '0' || *p > '9') fail("expected integer");
    int64_t v = 0;
    while (p < e && *p >= '0' && *p <= '9') v = v * 10 + (*p++ - '0');
    return neg ? -v : v;
  }
  // skip any JSON value (used for unknown keys)
  void skip() {
    ws();
    if (p >= e) fail("unexpected end");
    if (*p == '"') { str(); return; }
    if (*p == '{') {
      ++p;
      if (eat('}')) return;
      do { str(); expect(':'); skip(); } while (eat(','));
      expect('}');
      return;
    }
    if (*p == '[') {
      ++p;
      if (eat(']')) return;
      do { skip(); } while (eat(','));
      expect(']');
      return;
    }
    while (p < e && *p != ',' && *p != '}' && *p != ']') ++p;
  }
};

}  // namespace

SafeTensors::SafeTensors(const std::string& path) : file_(std::make_shared<MappedFile>(path)) {
  const uint8_t* b = file_->data();
  size_t n = file_->size();
  if (n < 8) throw std::runtime_error("safetensors: file too small " + path);
  uint64_t hlen = 0;
  for (int i = 7; i >= 0; --i) hlen = (hlen << 8) | b[i];
  if (hlen > n - 8 || hlen > (uint64_t(100) << 20)) throw std::runtime_error("safetensors: bad header length");
  data_off_ = 8 + hlen;
  const uint64_t data_len = n - data_off_;
  Json j{reinterpret_cast<const char*>(b + 8), reinterpret_cast<const char*>(b + 8 + hlen)};
  j.expect('{');
  if (!j.eat('}')) {
    do {
      std::string key = j.str();
      j.expect(':');
      if (key == "__metadata__") {
        j.expect('{');
        if (!j.eat('}')) {
          do {
            std::string k = j.str();
            j.expect(':');
            j.ws();
            if (j.p < j.e && *j.p == '"') meta_[k] = j.str();
            else j.skip();
          } while (j.eat(','));
          j.expect('}');
        }
        continue;
      }
      TensorInfo ti;
      bool have_off = false;
      j.expect('{');
      if (!j.eat('}')) {
        do {
          std::string f = j.str();
          j.expect(':');
          if (f == "dtype") {
            ti.dtype = j.str();
          } else if (f == "shape") {
            j.expect('[');
            if (!j.eat(']')) {
              do { ti.shape.push_back(j.integer()); } while (j.eat(','));
              j.expect(']');
            }
          } else if (f == "data_offsets") {
            j.expect('[');
            int64_t a = j.integer();
            j.expect(',');
            int64_t c = j.integer();
            j.expect(']');
            if (a < 0 || c < a || uint64_t(c) > data_len) throw std::runtime_error("safetensors: tensor " + key + " out of range");
            ti.begin = uint64_t(a);
            ti.end = uint64_t(c);
            have_off = true;
          } else {
            j.skip();
          }
        } while (j.eat(','));
        j.expect('}');
      }
      if (!have_off || ti.dtype.empty()) throw std::runtime_error("safetensors: incomplete entry " + key);
      order_.push_back(key);
      tensors_[key] = std::move(ti);
    } while (j.eat(','));
    j.expect('}');
  }
}

const TensorInfo& SafeTensors::info(const std::string& name) const {
  auto it = tensors_.find(name);
  if (it == tensors_.end()) throw std::out_of_range("safetensors: no tensor " + name);
  return it->second;
}

uint8_t* SafeTensors::tensor_ptr(const std::string& name) const {
  return file_->data() + data_off_ + info(name).begin;
}

void SafeTensors::copy_many(const std::vector<std::pair<std::string, uint8_t*>>& dst, int threads) const {
  struct Job { const uint8_t* src; uint8_t* dst; size_t n; };
  std::vector<Job> jobs;
  constexpr size_t SLICE = size_t(8) << 20;   // split big tensors so threads stay balanced
  for (auto& d : dst) {
    const TensorInfo& ti = info(d.first);
    const uint8_t* s = file_->data() + data_off_ + ti.begin;
    size_t n = ti.end - ti.begin;
    for (size_t o = 0; o < n; o += SLICE) jobs.push_back({s + o, d.second + o, std::min(SLICE, n - o)});
  }
  threads = std::max(1, std::min<int>(threads, int(jobs.size())));
  std::atomic<size_t> next{0};
  auto work = [&] {
    for (size_t i = next++; i < jobs.size(); i = next++) std::memcpy(jobs[i].dst, jobs[i].src, jobs[i].n);
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
}

std::string json_escape(const std::string& s) {
  std::string o;
  o.reserve(s.size() + 2);
  for (unsigned char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      case '\b': o += "\\b"; break;
      case '\f': o += "\\f"; break;
      default:
        if (c < 0x20) {
          char buf[8];
          std::snprintf(buf, sizeof(buf), "\\u%04x", c);
          o += buf;
        } else {
          o += char(c);
        }
    }
  }
  return o;
}

void save_safetensors(const std::string& path, const std::vector<SaveItem>& items,
                      const std::map<std::string, std::string>& metadata) {
  std::string h = "{";
  bool first = true;
  if (!metadata.empty()) {
    h += "\"__metadata__\":{";
    bool f2 = true;
    for (auto& kv : metadata) {
      if (!f2) h += ",";
      f2 = false;
      h += "\"" + json_escape(kv.first) + "\":\"" + json_escape(kv.second) + "\"";
    }
    h += "}";
    first = false;
  }
  uint64_t off = 0;
  for (auto& it : items) {
    if (!first) h += ",";
    first = false;
    h += "\"" + json_escape(it.name) + "\":{\"dtype\":\"" + it.dtype + "\",\"shape\":[";
    for (size_t i = 0; i < it.shape.size(); ++i) {
      if (i) h += ",";
      h += std::to_string(it.shape[i]);
    }
    h += "],\"data_offsets\":[" + std::to_string(off) + "," + std::to_string(off + it.bytes.size()) + "]}";
    off += it.bytes.size();
  }
  h += "}";
  while (h.size() % 8) h += ' ';
  std::string tmp = path + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) throw std::runtime_error("safetensors: cannot write " + path);
  uint64_t hl = h.size();
  uint8_t le[8];
  for (int i = 0; i < 8; ++i) le[i] = uint8_t(hl >> (8 * i));
  bool ok = std::fwrite(le, 1, 8, f) == 8 && std::fwrite(h.data(), 1, h.size(), f) == h.size();
  for (auto& it : items)
    ok = ok && (it.bytes.empty() || std::fwrite(it.bytes.data(), 1, it.bytes.size(), f) == it.bytes.size());
  ok = (std::fclose(f) == 0) && ok;
  if (!ok || std::rename(tmp.c_str(), path.c_str()) != 0) {
    std::remove(tmp.c_str());
    throw std::runtime_error("safetensors: write failed " + path);
  }
}

}  // namespace cgs
