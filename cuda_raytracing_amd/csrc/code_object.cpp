// code_object.cpp — kernel resource figures from an AMDGPU code object's metadata note (see code_object.h).
#include "code_object.h"

#include <cstring>
#include <map>
#include <memory>

namespace rt {
namespace {

// ---- a minimal msgpack reader (the subset the AMDGPU metadata uses: maps, arrays, strings, ints, bools, floats) ----
struct Value {
  enum Kind { NIL, BOOL, INT, FLOAT, STR, ARR, MAP } kind = NIL;
  int64_t i = 0;
  double f = 0;
  std::string s;
  std::vector<Value> arr;
  std::vector<std::pair<Value, Value>> map;
  const Value *get(const char *key) const {
    for (const auto &kv : map)
      if (kv.first.kind == STR && kv.first.s == key) return &kv.second;
    return nullptr;
  }
};

struct Reader {
  const uint8_t *p, *end;
  bool ok = true;
  uint64_t be(int n) {
    if (end - p < n) { ok = false; p = end; return 0; }
    uint64_t v = 0;
    for (int k = 0; k < n; ++k) v = (v << 8) | p[k];
    p += n;
    return v;
  }
  bool take(size_t n, std::string *s) {
    if (static_cast<size_t>(end - p) < n) { ok = false; p = end; return false; }
    if (s) s->assign(reinterpret_cast<const char *>(p), n);
    p += n;
    return true;
  }
  bool read(Value *v, int depth = 0) {
    if (!ok || p >= end || depth > 32) { ok = false; return false; }
    const uint8_t t = *p++;
    if (t <= 0x7f) { v->kind = Value::INT; v->i = t; return true; }
    if (t >= 0xe0) { v->kind = Value::INT; v->i = static_cast<int8_t>(t); return true; }
    if ((t & 0xf0) == 0x80) return read_map(v, t & 0x0f, depth);
    if ((t & 0xf0) == 0x90) return read_arr(v, t & 0x0f, depth);
    if ((t & 0xe0) == 0xa0) { v->kind = Value::STR; return take(t & 0x1f, &v->s); }
    switch (t) {
      case 0xc0: v->kind = Value::NIL; return true;
      case 0xc2: case 0xc3: v->kind = Value::BOOL; v->i = t == 0xc3; return true;
      case 0xc4: case 0xc5: case 0xc6: { const uint64_t n = be(1 << (t - 0xc4)); return take(n, nullptr); }
      case 0xc7: case 0xc8: case 0xc9: { const uint64_t n = be(1 << (t - 0xc7)); be(1); return take(n, nullptr); }
      case 0xca: { uint32_t u = static_cast<uint32_t>(be(4)); float f; std::memcpy(&f, &u, 4); v->kind = Value::FLOAT; v->f = f; return ok; }
      case 0xcb: { uint64_t u = be(8); double d; std::memcpy(&d, &u, 8); v->kind = Value::FLOAT; v->f = d; return ok; }
      case 0xcc: case 0xcd: case 0xce: case 0xcf: v->kind = Value::INT; v->i = static_cast<int64_t>(be(1 << (t - 0xcc))); return ok;
      case 0xd0: v->kind = Value::INT; v->i = static_cast<int8_t>(be(1)); return ok;
      case 0xd1: v->kind = Value::INT; v->i = static_cast<int16_t>(be(2)); return ok;
      case 0xd2: v->kind = Value::INT; v->i = static_cast<int32_t>(be(4)); return ok;
      case 0xd3: v->kind = Value::INT; v->i = static_cast<int64_t>(be(8)); return ok;
      case 0xd4: case 0xd5: case 0xd6: case 0xd7: case 0xd8: be(1); return take(1u << (t - 0xd4), nullptr);
      case 0xd9: case 0xda: case 0xdb: { const uint64_t n = be(1 << (t - 0xd9)); v->kind = Value::STR; return take(n, &v->s); }
      case 0xdc: case 0xdd: return read_arr(v, be(t == 0xdc ? 2 : 4), depth);
      case 0xde: case 0xdf: return read_map(v, be(t == 0xde ? 2 : 4), depth);
      default: ok = false; return false;
    }
  }
  bool read_arr(Value *v, uint64_t n, int depth) {
    v->kind = Value::ARR;
    if (n > static_cast<uint64_t>(end - p)) { ok = false; return false; }   // each element takes >= 1 byte
    v->arr.resize(n);
    for (auto &e : v->arr) if (!read(&e, depth + 1)) return false;
    return true;
  }
  bool read_map(Value *v, uint64_t n, int depth) {
    v->kind = Value::MAP;
    if (n > static_cast<uint64_t>(end - p) / 2) { ok = false; return false; }
    v->map.resize(n);
    for (auto &kv : v->map) if (!read(&kv.first, depth + 1) || !read(&kv.second, depth + 1)) return false;
    return true;
  }
};

int32_t int_of(const Value &m, const char *key) {
  const Value *v = m.get(key);
  return v && v->kind == Value::INT ? static_cast<int32_t>(v->i) : -1;
}

template <class T>
bool rd(const std::vector<char> &b, uint64_t off, T *out) {
  if (off > b.size() || b.size() - off < sizeof(T)) return false;
  std::memcpy(out, b.data() + off, sizeof(T));
  return true;
}

}  // namespace

bool code_object_kernels(const std::vector<char> &co, std::vector<KernelMeta> *out, std::string *compiler) {
  out->clear();
  if (compiler) compiler->clear();
  // ELF64 little-endian, EM_AMDGPU (224)
  if (co.size() < 64 || std::memcmp(co.data(), "\x7f" "ELF", 4) != 0 || co[4] != 2 || co[5] != 1) return false;
  uint16_t machine = 0, shentsize = 0, shnum = 0, shstrndx = 0;
  uint64_t shoff = 0;
  if (!rd(co, 18, &machine) || machine != 224 || !rd(co, 40, &shoff) || !rd(co, 58, &shentsize) || !rd(co, 60, &shnum) ||
      !rd(co, 62, &shstrndx) || shentsize < 64)
    return false;
  struct Sec { uint32_t name, type; uint64_t off, size; };
  std::vector<Sec> secs;
  for (uint16_t k = 0; k < shnum; ++k) {
    const uint64_t h = shoff + static_cast<uint64_t>(k) * shentsize;
    Sec s{};
    if (!rd(co, h, &s.name) || !rd(co, h + 4, &s.type) || !rd(co, h + 24, &s.off) || !rd(co, h + 32, &s.size)) return false;
    if (s.type == 8 /* SHT_NOBITS: no file bytes (.bss, .relro_padding) */ || s.type == 0) s.size = 0;
    if (s.off > co.size() || co.size() - s.off < s.size) return false;
    secs.push_back(s);
  }
  auto sec_name = [&](const Sec &s) -> std::string {
    if (shstrndx >= secs.size()) return "";
    const Sec &t = secs[shstrndx];
    if (s.name >= t.size) return "";
    const char *b = co.data() + t.off + s.name;
    return std::string(b, strnlen(b, t.size - s.name));
  };
  bool found = false;
  for (const Sec &s : secs) {
    const std::string nm = sec_name(s);
    if (compiler && nm == ".comment" && compiler->empty()) {
      // NUL-separated identification strings; keep the compiler's
      const char *b = co.data() + s.off;
      for (uint64_t k = 0; k < s.size;) {
        const std::string str(b + k, strnlen(b + k, s.size - k));
        if (str.find("clang version") != std::string::npos) { *compiler = str; break; }
        k += str.size() + 1;
      }
    }
    if (s.type != 7 /* SHT_NOTE */) continue;
    for (uint64_t k = s.off; k + 12 <= s.off + s.size;) {
      uint32_t namesz = 0, descsz = 0, type = 0;
      rd(co, k, &namesz); rd(co, k + 4, &descsz); rd(co, k + 8, &type);
      const uint64_t name_off = k + 12, desc_off = name_off + ((namesz + 3u) & ~3u);
      const uint64_t next = desc_off + ((descsz + 3u) & ~3ull);
      if (next > s.off + s.size) break;
      if (type == 32 /* NT_AMDGPU_METADATA */ && namesz >= 6 && std::memcmp(co.data() + name_off, "AMDGPU", 6) == 0) {
        Reader r{reinterpret_cast<const uint8_t *>(co.data() + desc_off), reinterpret_cast<const uint8_t *>(co.data() + desc_off + descsz)};
        Value root;
        if (r.read(&root) && root.kind == Value::MAP) {
          const Value *ks = root.get("amdhsa.kernels");
          if (ks && ks->kind == Value::ARR) {
            for (const Value &kd : ks->arr) {
              if (kd.kind != Value::MAP) continue;
              KernelMeta m;
              if (const Value *n = kd.get(".name"); n && n->kind == Value::STR) m.name = n->s;
              m.vgprs = int_of(kd, ".vgpr_count");
              m.agprs = int_of(kd, ".agpr_count");
              m.sgprs = int_of(kd, ".sgpr_count");
              m.scratch = int_of(kd, ".private_segment_fixed_size");
              m.vgpr_spills = int_of(kd, ".vgpr_spill_count");
              m.sgpr_spills = int_of(kd, ".sgpr_spill_count");
              m.lds = int_of(kd, ".group_segment_fixed_size");
              out->push_back(m);
            }
            found = true;
          }
        }
      }
      k = next;
    }
  }
  return found;
}

bool code_object_kernel(const std::vector<char> &co, const std::string &name, KernelMeta *out, std::string *compiler) {
  std::vector<KernelMeta> all;
  if (!code_object_kernels(co, &all, compiler)) return false;
  for (const KernelMeta &m : all)
    if (m.name == name) { *out = m; return true; }
  return false;
}

}  // namespace rt
