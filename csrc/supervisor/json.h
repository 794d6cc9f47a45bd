// Minimal JSON value + parser + writer for the supervisor's spec/state files.
#pragma once
#include <stdint.h>
#include <stdio.h>

#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace tpi {
namespace json {

struct Value {
  enum Type { NUL, BOOL, NUM, STR, ARR, OBJ } type = NUL;
  bool b = false;
  double n = 0;
  std::string s;
  std::vector<Value> a;
  std::map<std::string, Value> o;

  bool has(const std::string& k) const { return type == OBJ && o.count(k); }
  const Value& operator[](const std::string& k) const {
    static Value null_value;
    if (type != OBJ) return null_value;
    auto it = o.find(k);
    return it == o.end() ? null_value : it->second;
  }
  std::string str(const std::string& dflt = "") const { return type == STR ? s : dflt; }
  double num(double dflt = 0) const {
    return type == NUM ? n : type == BOOL ? (b ? 1 : 0) : dflt;
  }
  bool boolean(bool dflt = false) const { return type == BOOL ? b : type == NUM ? n != 0 : dflt; }
};

class Parser {
 public:
  explicit Parser(const std::string& text) : t_(text) {}
  Value parse() {
    Value v = value();
    ws();
    if (i_ != t_.size()) fail("trailing characters");
    return v;
  }

 private:
  const std::string& t_;
  size_t i_ = 0;
  [[noreturn]] void fail(const char* what) {
    throw std::runtime_error(std::string("json: ") + what + " at " + std::to_string(i_));
  }
  void ws() {
    while (i_ < t_.size() && (t_[i_] == ' ' || t_[i_] == '\n' || t_[i_] == '\r' || t_[i_] == '\t'))
      ++i_;
  }
  bool lit(const char* w) {
    size_t n = strlen_(w);
    if (t_.compare(i_, n, w) == 0) {
      i_ += n;
      return true;
    }
    return false;
  }
  static size_t strlen_(const char* s) {
    size_t n = 0;
    while (s[n]) ++n;
    return n;
  }
  static void utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) {
      out += (char)cp;
    } else if (cp < 0x800) {
      out += (char)(0xC0 | (cp >> 6));
      out += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      out += (char)(0xE0 | (cp >> 12));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    } else {
      out += (char)(0xF0 | (cp >> 18));
      out += (char)(0x80 | ((cp >> 12) & 0x3F));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    }
  }
  uint32_t hex4() {
    if (i_ + 4 > t_.size()) fail("bad \\u escape");
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {
      char c = t_[i_++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad hex digit");
    }
    return v;
  }
  std::string string() {
    if (t_[i_] != '"') fail("expected string");
    ++i_;
    std::string out;
    while (i_ < t_.size() && t_[i_] != '"') {
      char c = t_[i_++];
      if (c != '\\') {
        out += c;
        continue;
      }
      if (i_ >= t_.size()) fail("bad escape");
      char e = t_[i_++];
      switch (e) {
        case '"': out += '"'; break;
        case '\\': out += '\\'; break;
        case '/': out += '/'; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'n': out += '\n'; break;
        case 'r': out += '\r'; break;
        case 't': out += '\t'; break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && t_.compare(i_, 2, "\\u") == 0) {
            i_ += 2;
            uint32_t lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          utf8(out, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    if (i_ >= t_.size()) fail("unterminated string");
    ++i_;
    return out;
  }
  Value value() {
    ws();
    if (i_ >= t_.size()) fail("unexpected end");
    Value v;
    char c = t_[i_];
    if (c == '{') {
      v.type = Value::OBJ;
      ++i_;
      ws();
      if (t_[i_] == '}') {
        ++i_;
        return v;
      }
      for (;;) {
        ws();
        std::string k = string();
        ws();
        if (t_[i_++] != ':') fail("expected ':'");
        v.o[k] = value();
        ws();
        if (t_[i_] == ',') {
          ++i_;
          continue;
        }
        if (t_[i_] == '}') {
          ++i_;
          return v;
        }
        fail("expected ',' or '}'");
      }
    }
    if (c == '[') {
      v.type = Value::ARR;
      ++i_;
      ws();
      if (t_[i_] == ']') {
        ++i_;
        return v;
      }
      for (;;) {
        v.a.push_back(value());
        ws();
        if (t_[i_] == ',') {
          ++i_;
          continue;
        }
        if (t_[i_] == ']') {
          ++i_;
          return v;
        }
        fail("expected ',' or ']'");
      }
    }
    if (c == '"') {
      v.type = Value::STR;
      v.s = string();
      return v;
    }
    if (lit("true")) {
      v.type = Value::BOOL;
      v.b = true;
      return v;
    }
    if (lit("false")) {
      v.type = Value::BOOL;
      return v;
    }
    if (lit("null")) return v;
    size_t start = i_;
    while (i_ < t_.size() && (isdigit((unsigned char)t_[i_]) || t_[i_] == '-' || t_[i_] == '+' ||
                              t_[i_] == '.' || t_[i_] == 'e' || t_[i_] == 'E'))
      ++i_;
    if (start == i_) fail("unexpected character");
    v.type = Value::NUM;
    v.n = strtod(t_.substr(start, i_ - start).c_str(), nullptr);
    return v;
  }
};

inline Value parse(const std::string& text) { return Parser(text).parse(); }

inline std::string quote(const std::string& s) {
  std::string out = "\"";
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      default:
        if (c < 0x20) {
          char buf[8];
          snprintf(buf, sizeof(buf), "\\u%04x", c);
          out += buf;
        } else {
          out += (char)c;
        }
    }
  }
  return out + "\"";
}

}  // namespace json
}  // namespace tpi
