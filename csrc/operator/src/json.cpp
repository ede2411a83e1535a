#include "pto/json.hpp"

#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>

namespace pto {

// ----------------------------------------------------------------- JsonObject
JsonObject::JsonObject(const JsonObject& o) : items_(o.items_) {}
JsonObject& JsonObject::operator=(const JsonObject& o) {
  items_ = o.items_;
  return *this;
}
JsonObject::~JsonObject() = default;

Json* JsonObject::find(const std::string& k) {
  for (auto& it : items_)
    if (it.first == k) return &it.second;
  return nullptr;
}
const Json* JsonObject::find(const std::string& k) const {
  for (const auto& it : items_)
    if (it.first == k) return &it.second;
  return nullptr;
}
Json& JsonObject::operator[](const std::string& k) {
  if (Json* j = find(k)) return *j;
  items_.emplace_back(k, Json());
  return items_.back().second;
}
bool JsonObject::erase(const std::string& k) {
  for (auto it = items_.begin(); it != items_.end(); ++it) {
    if (it->first == k) {
      items_.erase(it);
      return true;
    }
  }
  return false;
}
bool JsonObject::operator==(const JsonObject& o) const {
  if (items_.size() != o.items_.size()) return false;
  for (const auto& it : items_) {
    const Json* v = o.find(it.first);
    if (!v || !(*v == it.second)) return false;
  }
  return true;
}

// ----------------------------------------------------------------------- Json
void Json::copy_from(const Json& o) {
  type_ = o.type_;
  b_ = o.b_;
  i_ = o.i_;
  d_ = o.d_;
  s_.reset();
  a_.reset();
  o_.reset();
  if (o.s_) s_ = std::make_shared<std::string>(*o.s_);
  if (o.a_) a_ = std::make_shared<JsonArray>(*o.a_);
  if (o.o_) o_ = std::make_shared<JsonObject>(*o.o_);
}

bool Json::as_bool() const {
  if (type_ != Type::Bool) throw JsonError("not a bool");
  return b_;
}
int64_t Json::as_int() const {
  if (type_ == Type::Int) return i_;
  if (type_ == Type::Double) return (int64_t)d_;
  throw JsonError("not a number");
}
double Json::as_double() const {
  if (type_ == Type::Double) return d_;
  if (type_ == Type::Int) return (double)i_;
  throw JsonError("not a number");
}
const std::string& Json::as_string() const {
  if (type_ != Type::String) throw JsonError("not a string");
  return *s_;
}
const JsonArray& Json::as_array() const {
  if (type_ != Type::Array) throw JsonError("not an array");
  return *a_;
}
JsonArray& Json::as_array() {
  if (type_ == Type::Null) *this = Json::array();
  if (type_ != Type::Array) throw JsonError("not an array");
  return *a_;
}
const JsonObject& Json::as_object() const {
  if (type_ != Type::Object) throw JsonError("not an object");
  return *o_;
}
JsonObject& Json::as_object() {
  if (type_ == Type::Null) *this = Json::object();
  if (type_ != Type::Object) throw JsonError("not an object");
  return *o_;
}

Json& Json::operator[](const std::string& k) { return as_object()[k]; }
const Json* Json::get(const std::string& k) const {
  if (type_ != Type::Object) return nullptr;
  return o_->find(k);
}
Json* Json::get(const std::string& k) {
  if (type_ != Type::Object) return nullptr;
  return o_->find(k);
}
bool Json::erase(const std::string& k) {
  if (type_ != Type::Object) return false;
  return o_->erase(k);
}
Json& Json::operator[](size_t i) { return as_array().at(i); }
const Json& Json::operator[](size_t i) const { return as_array().at(i); }
void Json::push_back(Json v) { as_array().push_back(std::move(v)); }
size_t Json::size() const {
  if (type_ == Type::Array) return a_->size();
  if (type_ == Type::Object) return o_->size();
  return 0;
}

const Json* Json::path(std::initializer_list<const char*> keys) const {
  const Json* cur = this;
  for (const char* k : keys) {
    cur = cur->get(k);
    if (!cur) return nullptr;
  }
  return cur;
}
Json* Json::path(std::initializer_list<const char*> keys) {
  Json* cur = this;
  for (const char* k : keys) {
    cur = cur->get(k);
    if (!cur) return nullptr;
  }
  return cur;
}
std::string Json::str_or(const std::string& k, const std::string& def) const {
  const Json* v = get(k);
  return (v && v->is_string()) ? v->as_string() : def;
}
int64_t Json::int_or(const std::string& k, int64_t def) const {
  const Json* v = get(k);
  return (v && v->is_number()) ? v->as_int() : def;
}
bool Json::bool_or(const std::string& k, bool def) const {
  const Json* v = get(k);
  return (v && v->is_bool()) ? v->as_bool() : def;
}

bool Json::operator==(const Json& o) const {
  if (is_number() && o.is_number()) {
    if (type_ == Type::Int && o.type_ == Type::Int) return i_ == o.i_;
    return as_double() == o.as_double();
  }
  if (type_ != o.type_) return false;
  switch (type_) {
    case Type::Null: return true;
    case Type::Bool: return b_ == o.b_;
    case Type::String: return *s_ == *o.s_;
    case Type::Array: return *a_ == *o.a_;
    case Type::Object: return *o_ == *o.o_;
    default: return false;
  }
}

std::string json_escape(const std::string& s) {
  std::string out;
  out.reserve(s.size() + 2);
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      default:
        if (c < 0x20) {
          char buf[8];
          std::snprintf(buf, sizeof buf, "\\u%04x", c);
          out += buf;
        } else {
          out += (char)c;
        }
    }
  }
  return out;
}

void Json::dump_to(std::string& out, int indent, int depth) const {
  auto nl = [&](int d) {
    if (indent < 0) return;
    out += '\n';
    out.append((size_t)(indent * d), ' ');
  };
  switch (type_) {
    case Type::Null: out += "null"; break;
    case Type::Bool: out += b_ ? "true" : "false"; break;
    case Type::Int: out += std::to_string(i_); break;
    case Type::Double: {
      if (!std::isfinite(d_)) {
        out += "null";
        break;
      }
      char buf[32];
      std::snprintf(buf, sizeof buf, "%.17g", d_);
      out += buf;
      break;
    }
    case Type::String:
      out += '"';
      out += json_escape(*s_);
      out += '"';
      break;
    case Type::Array: {
      out += '[';
      bool first = true;
      for (const auto& v : *a_) {
        if (!first) out += ',';
        first = false;
        nl(depth + 1);
        v.dump_to(out, indent, depth + 1);
      }
      if (!a_->empty()) nl(depth);
      out += ']';
      break;
    }
    case Type::Object: {
      out += '{';
      bool first = true;
      for (const auto& kv : *o_) {
        if (!first) out += ',';
        first = false;
        nl(depth + 1);
        out += '"';
        out += json_escape(kv.first);
        out += indent < 0 ? "\":" : "\": ";
        kv.second.dump_to(out, indent, depth + 1);
      }
      if (!o_->empty()) nl(depth);
      out += '}';
      break;
    }
  }
}

std::string Json::dump(int indent) const {
  std::string out;
  dump_to(out, indent, 0);
  return out;
}

// --------------------------------------------------------------------- parser
namespace {
struct Parser {
  const char* p;
  const char* end;
  int depth = 0;

  [[noreturn]] void fail(const char* what) {
    throw JsonError(std::string("json parse error: ") + what);
  }
  void ws() {
    while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  }
  bool lit(const char* s) {
    size_t n = std::strlen(s);
    if ((size_t)(end - p) >= n && std::memcmp(p, s, n) == 0) {
      p += n;
      return true;
    }
    return false;
  }
  static void put_utf8(std::string& out, uint32_t cp) {
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
    if (end - p < 4) fail("short \\u escape");
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = *p++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
      else fail("bad \\u escape");
    }
    return v;
  }
  std::string str() {
    if (p >= end || *p != '"') fail("expected string");
    ++p;
    std::string out;
    while (true) {
      if (p >= end) fail("unterminated string");
      char c = *p++;
      if (c == '"') break;
      if ((unsigned char)c < 0x20) fail("control character in string");
      if (c != '\\') {
        out += c;
        continue;
      }
      if (p >= end) fail("bad escape");
      char e = *p++;
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
          if (cp >= 0xD800 && cp <= 0xDBFF) {
            if (end - p >= 6 && p[0] == '\\' && p[1] == 'u') {
              p += 2;
              uint32_t lo = hex4();
              if (lo < 0xDC00 || lo > 0xDFFF) fail("bad surrogate pair");
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            } else {
              fail("lone surrogate");
            }
          }
          put_utf8(out, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    return out;
  }
  Json number() {
    const char* s = p;
    bool is_float = false;
    if (p < end && *p == '-') ++p;
    if (p >= end || !(*p >= '0' && *p <= '9')) fail("bad number");
    while (p < end && *p >= '0' && *p <= '9') ++p;
    if (p < end && *p == '.') {
      is_float = true;
      ++p;
      if (p >= end || !(*p >= '0' && *p <= '9')) fail("bad fraction");
      while (p < end && *p >= '0' && *p <= '9') ++p;
    }
    if (p < end && (*p == 'e' || *p == 'E')) {
      is_float = true;
      ++p;
      if (p < end && (*p == '+' || *p == '-')) ++p;
      if (p >= end || !(*p >= '0' && *p <= '9')) fail("bad exponent");
      while (p < end && *p >= '0' && *p <= '9') ++p;
    }
    std::string tok(s, p);
    if (!is_float) {
      errno = 0;
      char* e = nullptr;
      long long v = std::strtoll(tok.c_str(), &e, 10);
      if (errno == 0) return Json(v);
    }
    return Json(std::strtod(tok.c_str(), nullptr));
  }
  Json value() {
    ws();
    if (p >= end) fail("unexpected end");
    if (++depth > 512) fail("nesting too deep");
    Json out;
    char c = *p;
    if (c == '{') {
      ++p;
      JsonObject obj;
      ws();
      if (p < end && *p == '}') {
        ++p;
      } else {
        while (true) {
          ws();
          std::string k = str();
          ws();
          if (p >= end || *p != ':') fail("expected ':'");
          ++p;
          obj[k] = value();
          ws();
          if (p < end && *p == ',') {
            ++p;
            continue;
          }
          if (p < end && *p == '}') {
            ++p;
            break;
          }
          fail("expected ',' or '}'");
        }
      }
      out = Json(std::move(obj));
    } else if (c == '[') {
      ++p;
      JsonArray arr;
      ws();
      if (p < end && *p == ']') {
        ++p;
      } else {
        while (true) {
          arr.push_back(value());
          ws();
          if (p < end && *p == ',') {
            ++p;
            continue;
          }
          if (p < end && *p == ']') {
            ++p;
            break;
          }
          fail("expected ',' or ']'");
        }
      }
      out = Json(std::move(arr));
    } else if (c == '"') {
      out = Json(str());
    } else if (lit("true")) {
      out = Json(true);
    } else if (lit("false")) {
      out = Json(false);
    } else if (lit("null")) {
      out = Json();
    } else {
      out = number();
    }
    --depth;
    return out;
  }
};
}  // namespace

Json Json::parse(const std::string& text) {
  Parser ps{text.data(), text.data() + text.size()};
  Json v = ps.value();
  ps.ws();
  if (ps.p != ps.end) ps.fail("trailing characters");
  return v;
}

void json_merge_patch(Json& target, const Json& patch) {
  if (!patch.is_object()) {
    target = patch;
    return;
  }
  if (!target.is_object()) target = Json::object();
  for (const auto& kv : patch.as_object()) {
    if (kv.second.is_null()) {
      target.erase(kv.first);
    } else {
      json_merge_patch(target[kv.first], kv.second);
    }
  }
}

}  // namespace pto
