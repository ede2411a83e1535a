// Minimal JSON value for the PyTorchJob operator: Kubernetes objects are JSON
// documents, and most of a Pod/Service template is opaque to the controller, so
// the operator keeps objects as `Json` and reads/writes the fields it reasons about.
//
// * objects preserve insertion order (stable, diff-friendly manifests);
// * integers are kept as int64 (resourceVersion-style numbers, ports, counts),
//   other numbers as double;
// * parse() is strict RFC 8259 (UTF-8 passthrough, \uXXXX incl. surrogates);
// * dump() emits compact JSON; dump(2) pretty-prints.
#pragma once

#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace pto {

class Json;
using JsonArray = std::vector<Json>;

class JsonObject {
 public:
  using Item = std::pair<std::string, Json>;
  JsonObject() = default;
  JsonObject(const JsonObject&);
  JsonObject& operator=(const JsonObject&);
  JsonObject(JsonObject&&) noexcept = default;
  JsonObject& operator=(JsonObject&&) noexcept = default;
  ~JsonObject();

  Json* find(const std::string& k);
  const Json* find(const std::string& k) const;
  Json& operator[](const std::string& k);  // inserts null when absent
  bool contains(const std::string& k) const { return find(k) != nullptr; }
  bool erase(const std::string& k);
  size_t size() const { return items_.size(); }
  bool empty() const { return items_.empty(); }
  std::deque<Item>::iterator begin() { return items_.begin(); }
  std::deque<Item>::iterator end() { return items_.end(); }
  std::deque<Item>::const_iterator begin() const { return items_.begin(); }
  std::deque<Item>::const_iterator end() const { return items_.end(); }
  bool operator==(const JsonObject& o) const;  // order-insensitive

 private:
  std::deque<Item> items_;  // deque: inserting keeps pointers to other members valid
};

class JsonError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

class Json {
 public:
  enum class Type { Null, Bool, Int, Double, String, Array, Object };

  Json() : type_(Type::Null) {}
  Json(std::nullptr_t) : type_(Type::Null) {}
  Json(bool b) : type_(Type::Bool), b_(b) {}
  Json(int v) : type_(Type::Int), i_(v) {}
  Json(long v) : type_(Type::Int), i_(v) {}
  Json(long long v) : type_(Type::Int), i_(v) {}
  Json(unsigned v) : type_(Type::Int), i_(v) {}
  Json(double v) : type_(Type::Double), d_(v) {}
  Json(const char* s) : type_(Type::String), s_(std::make_shared<std::string>(s)) {}
  Json(std::string s) : type_(Type::String), s_(std::make_shared<std::string>(std::move(s))) {}
  Json(JsonArray a) : type_(Type::Array), a_(std::make_shared<JsonArray>(std::move(a))) {}
  Json(JsonObject o) : type_(Type::Object), o_(std::make_shared<JsonObject>(std::move(o))) {}

  Json(const Json& o) { copy_from(o); }
  Json& operator=(const Json& o) {
    if (this != &o) copy_from(o);
    return *this;
  }
  Json(Json&&) noexcept = default;
  Json& operator=(Json&&) noexcept = default;

  static Json object() { return Json(JsonObject()); }
  static Json array() { return Json(JsonArray()); }

  Type type() const { return type_; }
  bool is_null() const { return type_ == Type::Null; }
  bool is_bool() const { return type_ == Type::Bool; }
  bool is_int() const { return type_ == Type::Int; }
  bool is_number() const { return type_ == Type::Int || type_ == Type::Double; }
  bool is_string() const { return type_ == Type::String; }
  bool is_array() const { return type_ == Type::Array; }
  bool is_object() const { return type_ == Type::Object; }

  bool as_bool() const;
  int64_t as_int() const;
  double as_double() const;
  const std::string& as_string() const;
  const JsonArray& as_array() const;
  JsonArray& as_array();
  const JsonObject& as_object() const;
  JsonObject& as_object();

  // Object access.  operator[] on a null value turns it into an object.
  Json& operator[](const std::string& k);
  Json& operator[](const char* k) { return (*this)[std::string(k)]; }
  const Json* get(const std::string& k) const;  // nullptr when absent / not an object
  Json* get(const std::string& k);
  bool contains(const std::string& k) const { return get(k) != nullptr; }
  bool erase(const std::string& k);
  // Array access.
  Json& operator[](size_t i);
  const Json& operator[](size_t i) const;
  Json& operator[](int i) { return (*this)[(size_t)i]; }  // literal 0 must not mean (const char*)0
  const Json& operator[](int i) const { return (*this)[(size_t)i]; }
  void push_back(Json v);
  size_t size() const;

  // Path helpers: path("a", "b") -> value at a.b or nullptr.
  const Json* path(std::initializer_list<const char*> keys) const;
  Json* path(std::initializer_list<const char*> keys);
  // Defaults when absent / wrong type.
  std::string str_or(const std::string& k, const std::string& def = "") const;
  int64_t int_or(const std::string& k, int64_t def) const;
  bool bool_or(const std::string& k, bool def) const;

  std::string dump(int indent = -1) const;
  static Json parse(const std::string& text);  // throws JsonError

  bool operator==(const Json& o) const;
  bool operator!=(const Json& o) const { return !(*this == o); }

 private:
  void copy_from(const Json& o);
  void dump_to(std::string& out, int indent, int depth) const;

  Type type_ = Type::Null;
  bool b_ = false;
  int64_t i_ = 0;
  double d_ = 0.0;
  std::shared_ptr<std::string> s_;
  std::shared_ptr<JsonArray> a_;
  std::shared_ptr<JsonObject> o_;
};

std::string json_escape(const std::string& s);

// RFC 7386 JSON merge patch: apply `patch` onto `target` in place.
void json_merge_patch(Json& target, const Json& patch);

}  // namespace pto
