// Minimal JSON reader/writer used by the kbref oracle (test infrastructure only).
// Values keep object-key insertion order so fixture order is preserved.
#pragma once
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace kbjson {

struct Value {
  enum Kind { Null, Bool, Int, Double, String, Array, Object } kind = Null;
  bool b = false;
  int64_t i = 0;
  double d = 0;
  std::string s;
  std::vector<Value> arr;
  std::vector<std::pair<std::string, Value>> obj;

  bool is_null() const { return kind == Null; }
  bool is_obj() const { return kind == Object; }
  bool is_arr() const { return kind == Array; }
  bool is_str() const { return kind == String; }
  bool is_num() const { return kind == Int || kind == Double; }
  const Value* get(const std::string& k) const {
    if (kind != Object) return nullptr;
    for (auto& kv : obj)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  std::string str(const std::string& k, const std::string& def = "") const {
    const Value* v = get(k);
    if (!v || v->is_null()) return def;
    if (v->kind != String) throw std::runtime_error("json: field '" + k + "' is not a string");
    return v->s;
  }
  int64_t integer(const std::string& k, int64_t def = 0) const {
    const Value* v = get(k);
    if (!v || v->is_null()) return def;
    if (v->kind == Int) return v->i;
    if (v->kind == Double) return (int64_t)v->d;
    if (v->kind == Bool) return v->b ? 1 : 0;
    throw std::runtime_error("json: field '" + k + "' is not a number");
  }
  bool boolean(const std::string& k, bool def = false) const {
    const Value* v = get(k);
    if (!v || v->is_null()) return def;
    if (v->kind == Bool) return v->b;
    if (v->kind == Int) return v->i != 0;
    throw std::runtime_error("json: field '" + k + "' is not a bool");
  }
};

class Parser {
 public:
  explicit Parser(const std::string& t) : s_(t), p_(0) {}
  Value parse() {
    Value v = value();
    ws();
    if (p_ != s_.size()) fail("trailing characters");
    return v;
  }

 private:
  const std::string& s_;
  size_t p_;
  [[noreturn]] void fail(const char* m) {
    throw std::runtime_error(std::string("json parse error: ") + m + " at offset " + std::to_string(p_));
  }
  void ws() {
    while (p_ < s_.size() && (s_[p_] == ' ' || s_[p_] == '\n' || s_[p_] == '\t' || s_[p_] == '\r')) p_++;
  }
  Value value() {
    ws();
    if (p_ >= s_.size()) fail("unexpected end");
    char c = s_[p_];
    Value v;
    if (c == '{') {
      v.kind = Value::Object;
      p_++;
      ws();
      if (s_[p_] == '}') { p_++; return v; }
      for (;;) {
        ws();
        if (s_[p_] != '"') fail("expected key");
        std::string k = string_lit();
        ws();
        if (s_[p_] != ':') fail("expected ':'");
        p_++;
        v.obj.emplace_back(std::move(k), value());
        ws();
        if (s_[p_] == ',') { p_++; continue; }
        if (s_[p_] == '}') { p_++; break; }
        fail("expected ',' or '}'");
      }
    } else if (c == '[') {
      v.kind = Value::Array;
      p_++;
      ws();
      if (s_[p_] == ']') { p_++; return v; }
      for (;;) {
        v.arr.push_back(value());
        ws();
        if (s_[p_] == ',') { p_++; continue; }
        if (s_[p_] == ']') { p_++; break; }
        fail("expected ',' or ']'");
      }
    } else if (c == '"') {
      v.kind = Value::String;
      v.s = string_lit();
    } else if (s_.compare(p_, 4, "true") == 0) {
      v.kind = Value::Bool; v.b = true; p_ += 4;
    } else if (s_.compare(p_, 5, "false") == 0) {
      v.kind = Value::Bool; v.b = false; p_ += 5;
    } else if (s_.compare(p_, 4, "null") == 0) {
      p_ += 4;
    } else {
      size_t st = p_;
      bool flt = false;
      if (s_[p_] == '-') p_++;
      while (p_ < s_.size()) {
        char d = s_[p_];
        if (d >= '0' && d <= '9') { p_++; continue; }
        if (d == '.' || d == 'e' || d == 'E' || d == '+' || d == '-') { flt = true; p_++; continue; }
        break;
      }
      std::string num = s_.substr(st, p_ - st);
      if (num.empty() || num == "-") fail("bad number");
      if (flt) { v.kind = Value::Double; v.d = strtod(num.c_str(), nullptr); }
      else { v.kind = Value::Int; v.i = strtoll(num.c_str(), nullptr, 10); }
    }
    return v;
  }
  static void put_utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) o += (char)cp;
    else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) { o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F)); }
    else { o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 0x3F)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F)); }
  }
  std::string string_lit() {
    std::string o;
    p_++;  // opening quote
    while (p_ < s_.size() && s_[p_] != '"') {
      char c = s_[p_++];
      if (c != '\\') { o += c; continue; }
      char e = s_[p_++];
      switch (e) {
        case 'n': o += '\n'; break;
        case 't': o += '\t'; break;
        case 'r': o += '\r'; break;
        case 'b': o += '\b'; break;
        case 'f': o += '\f'; break;
        case 'u': {
          uint32_t cp = (uint32_t)strtoul(s_.substr(p_, 4).c_str(), nullptr, 16);
          p_ += 4;
          if (cp >= 0xD800 && cp < 0xDC00 && s_.compare(p_, 2, "\\u") == 0) {
            uint32_t lo = (uint32_t)strtoul(s_.substr(p_ + 2, 4).c_str(), nullptr, 16);
            p_ += 6;
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(o, cp);
          break;
        }
        default: o += e;
      }
    }
    if (p_ >= s_.size()) fail("unterminated string");
    p_++;
    return o;
  }
};

inline Value parse_file(const std::string& path) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("cannot open " + path);
  std::string buf;
  char tmp[1 << 16];
  size_t n;
  while ((n = fread(tmp, 1, sizeof tmp, f)) > 0) buf.append(tmp, n);
  fclose(f);
  return Parser(buf).parse();
}

inline std::string quote(const std::string& s) {
  std::string o = "\"";
  for (unsigned char c : s) {
    if (c == '"') o += "\\\"";
    else if (c == '\\') o += "\\\\";
    else if (c == '\n') o += "\\n";
    else if (c < 0x20) { char b[8]; snprintf(b, sizeof b, "\\u%04x", c); o += b; }
    else o += (char)c;
  }
  return o + "\"";
}

inline std::string num(double d) {
  char b[40];
  snprintf(b, sizeof b, "%.17g", d);
  return b;
}

}  // namespace kbjson
