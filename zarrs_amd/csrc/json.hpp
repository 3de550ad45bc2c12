// Minimal JSON reader for Zarr codec metadata (MetadataV3 {name, configuration} lists).
// Mirrors only what zarrs_metadata needs on this path: objects, arrays, strings, numbers, bools.
#pragma once
#include <cstdint>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace zgpu {

struct Json {
  enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
  bool b = false;
  double num = 0;
  bool is_int = false;
  int64_t i = 0;
  std::string s;
  std::vector<Json> arr;
  std::map<std::string, Json> obj;

  const Json *get(const std::string &k) const {
    if (kind != Obj) return nullptr;
    auto it = obj.find(k);
    return it == obj.end() ? nullptr : &it->second;
  }
  int64_t as_int() const {
    if (kind != Num) throw std::runtime_error("expected a number");
    return is_int ? i : (int64_t)num;
  }
  const std::string &as_str() const {
    if (kind != Str) throw std::runtime_error("expected a string");
    return s;
  }

  static Json parse(const std::string &text) {
    size_t p = 0;
    Json j = parse_value(text, p);
    skip_ws(text, p);
    if (p != text.size()) throw std::runtime_error("trailing characters in JSON");
    return j;
  }

 private:
  static void skip_ws(const std::string &t, size_t &p) {
    while (p < t.size() && (t[p] == ' ' || t[p] == '\n' || t[p] == '\t' || t[p] == '\r')) p++;
  }
  static std::string parse_string(const std::string &t, size_t &p) {
    if (t[p] != '"') throw std::runtime_error("expected '\"'");
    p++;
    std::string out;
    while (p < t.size() && t[p] != '"') {
      char c = t[p++];
      if (c == '\\') {
        if (p >= t.size()) break;
        char e = t[p++];
        switch (e) {
          case 'n': out += '\n'; break;
          case 't': out += '\t'; break;
          case 'r': out += '\r'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'u': {
            unsigned v = (unsigned)std::strtoul(t.substr(p, 4).c_str(), nullptr, 16);
            p += 4;
            if (v < 0x80) out += (char)v;
            else if (v < 0x800) { out += (char)(0xC0 | (v >> 6)); out += (char)(0x80 | (v & 0x3F)); }
            else { out += (char)(0xE0 | (v >> 12)); out += (char)(0x80 | ((v >> 6) & 0x3F)); out += (char)(0x80 | (v & 0x3F)); }
            break;
          }
          default: out += e;
        }
      } else {
        out += c;
      }
    }
    if (p >= t.size()) throw std::runtime_error("unterminated string");
    p++;
    return out;
  }
  static Json parse_value(const std::string &t, size_t &p) {
    skip_ws(t, p);
    if (p >= t.size()) throw std::runtime_error("unexpected end of JSON");
    Json j;
    char c = t[p];
    if (c == '{') {
      j.kind = Obj;
      p++;
      skip_ws(t, p);
      if (t[p] == '}') { p++; return j; }
      for (;;) {
        skip_ws(t, p);
        std::string k = parse_string(t, p);
        skip_ws(t, p);
        if (t[p] != ':') throw std::runtime_error("expected ':'");
        p++;
        j.obj[k] = parse_value(t, p);
        skip_ws(t, p);
        if (t[p] == ',') { p++; continue; }
        if (t[p] == '}') { p++; break; }
        throw std::runtime_error("expected ',' or '}'");
      }
    } else if (c == '[') {
      j.kind = Arr;
      p++;
      skip_ws(t, p);
      if (t[p] == ']') { p++; return j; }
      for (;;) {
        j.arr.push_back(parse_value(t, p));
        skip_ws(t, p);
        if (t[p] == ',') { p++; continue; }
        if (t[p] == ']') { p++; break; }
        throw std::runtime_error("expected ',' or ']'");
      }
    } else if (c == '"') {
      j.kind = Str;
      j.s = parse_string(t, p);
    } else if (t.compare(p, 4, "true") == 0) {
      j.kind = Bool; j.b = true; p += 4;
    } else if (t.compare(p, 5, "false") == 0) {
      j.kind = Bool; j.b = false; p += 5;
    } else if (t.compare(p, 4, "null") == 0) {
      j.kind = Null; p += 4;
    } else {
      size_t s0 = p;
      bool integral = true;
      if (t[p] == '-' || t[p] == '+') p++;
      while (p < t.size() && (isdigit((unsigned char)t[p]) || t[p] == '.' || t[p] == 'e' ||
                              t[p] == 'E' || t[p] == '-' || t[p] == '+')) {
        if (t[p] == '.' || t[p] == 'e' || t[p] == 'E') integral = false;
        p++;
      }
      if (p == s0) throw std::runtime_error("invalid JSON value");
      std::string tok = t.substr(s0, p - s0);
      j.kind = Num;
      j.num = std::strtod(tok.c_str(), nullptr);
      j.is_int = integral;
      if (integral) j.i = std::strtoll(tok.c_str(), nullptr, 10);
    }
    return j;
  }
};

}  // namespace zgpu
