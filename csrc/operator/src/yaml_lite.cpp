#include "pto/yaml_lite.hpp"

#include <cstdlib>
#include <vector>

namespace pto {
namespace {

struct Line {
  int indent;
  std::string text;  // content without indentation / trailing comment
};

std::string strip_comment(const std::string& s) {
  bool sq = false, dq = false;
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (c == '\'' && !dq) sq = !sq;
    else if (c == '"' && !sq && (i == 0 || s[i - 1] != '\\')) dq = !dq;
    else if (c == '#' && !sq && !dq && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '\t')) return s.substr(0, i);
  }
  return s;
}

std::string rtrim(std::string s) {
  while (!s.empty() && (s.back() == ' ' || s.back() == '\t' || s.back() == '\r')) s.pop_back();
  return s;
}
std::string trim(const std::string& s) {
  size_t a = 0;
  while (a < s.size() && (s[a] == ' ' || s[a] == '\t')) ++a;
  return rtrim(s.substr(a));
}

Json scalar(const std::string& raw);

// split a flow collection body on top-level commas
std::vector<std::string> split_flow(const std::string& body) {
  std::vector<std::string> out;
  int depth = 0;
  bool sq = false, dq = false;
  std::string cur;
  for (size_t i = 0; i < body.size(); ++i) {
    char c = body[i];
    if (c == '\'' && !dq) sq = !sq;
    else if (c == '"' && !sq && (i == 0 || body[i - 1] != '\\')) dq = !dq;
    if (!sq && !dq) {
      if (c == '[' || c == '{') ++depth;
      if (c == ']' || c == '}') --depth;
      if (c == ',' && depth == 0) {
        out.push_back(trim(cur));
        cur.clear();
        continue;
      }
    }
    cur += c;
  }
  if (!trim(cur).empty()) out.push_back(trim(cur));
  return out;
}

// index of the "key: value" colon outside quotes/brackets, or npos
size_t key_colon(const std::string& s) {
  bool sq = false, dq = false;
  int depth = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (c == '\'' && !dq) sq = !sq;
    else if (c == '"' && !sq && (i == 0 || s[i - 1] != '\\')) dq = !dq;
    if (sq || dq) continue;
    if (c == '[' || c == '{') ++depth;
    if (c == ']' || c == '}') --depth;
    if (c == ':' && depth == 0 && (i + 1 == s.size() || s[i + 1] == ' ')) return i;
  }
  return std::string::npos;
}

std::string unquote_key(const std::string& k) {
  std::string t = trim(k);
  if (t.size() >= 2 && ((t.front() == '"' && t.back() == '"') || (t.front() == '\'' && t.back() == '\'')))
    return scalar(t).as_string();
  return t;
}

Json scalar(const std::string& raw) {
  std::string s = trim(raw);
  if (s.empty() || s == "~" || s == "null" || s == "Null" || s == "NULL") return Json();
  if (s.front() == '[') {
    if (s.back() != ']') throw JsonError("yaml: unterminated flow sequence");
    Json a = Json::array();
    for (const auto& item : split_flow(s.substr(1, s.size() - 2))) a.push_back(scalar(item));
    return a;
  }
  if (s.front() == '{') {
    if (s.back() != '}') throw JsonError("yaml: unterminated flow mapping");
    Json o = Json::object();
    for (const auto& item : split_flow(s.substr(1, s.size() - 2))) {
      size_t c = key_colon(item);
      if (c == std::string::npos) throw JsonError("yaml: bad flow mapping entry");
      o[unquote_key(item.substr(0, c))] = scalar(item.substr(c + 1));
    }
    return o;
  }
  if (s.front() == '\'') {
    if (s.size() < 2 || s.back() != '\'') throw JsonError("yaml: unterminated single quote");
    std::string out;
    for (size_t i = 1; i + 1 < s.size(); ++i) {
      if (s[i] == '\'' && i + 2 < s.size() && s[i + 1] == '\'') {
        out += '\'';
        ++i;
      } else {
        out += s[i];
      }
    }
    return Json(out);
  }
  if (s.front() == '"') {
    if (s.size() < 2 || s.back() != '"') throw JsonError("yaml: unterminated double quote");
    return Json::parse(s);  // JSON string escapes are a subset of YAML's
  }
  if (s == "true" || s == "True" || s == "TRUE") return Json(true);
  if (s == "false" || s == "False" || s == "FALSE") return Json(false);
  // numbers
  char* end = nullptr;
  long long iv = std::strtoll(s.c_str(), &end, 10);
  if (end && *end == '\0') return Json(iv);
  double dv = std::strtod(s.c_str(), &end);
  if (end && *end == '\0' && s.find_first_of("0123456789") != std::string::npos) return Json(dv);
  return Json(s);
}

class YamlParser {
 public:
  explicit YamlParser(std::vector<Line> lines) : lines_(std::move(lines)) {}

  Json parse_document() {
    if (lines_.empty()) return Json();
    Json v = parse_block(lines_[0].indent);
    if (pos_ != lines_.size()) throw JsonError("yaml: unexpected indentation");
    return v;
  }

 private:
  bool is_seq_item(const std::string& t) const { return t == "-" || (t.size() >= 2 && t[0] == '-' && t[1] == ' '); }

  Json parse_block(int indent) {
    if (pos_ >= lines_.size()) return Json();
    if (is_seq_item(lines_[pos_].text)) return parse_seq(indent);
    return parse_map(indent);
  }

  Json parse_seq(int indent) {
    Json arr = Json::array();
    while (pos_ < lines_.size() && lines_[pos_].indent == indent && is_seq_item(lines_[pos_].text)) {
      const std::string& lt = lines_[pos_].text;
      size_t sp = 1;
      while (sp < lt.size() && lt[sp] == ' ') ++sp;
      std::string rest = trim(lt.substr(sp));
      const int item_col = indent + (int)sp;  // column of the first key of a mapping item
      ++pos_;
      if (rest.empty()) {
        if (pos_ < lines_.size() && lines_[pos_].indent > indent) arr.push_back(parse_block(lines_[pos_].indent));
        else arr.push_back(Json());
        continue;
      }
      size_t c = key_colon(rest);
      if (c != std::string::npos && rest.front() != '[' && rest.front() != '{' && rest.front() != '"' &&
          rest.front() != '\'') {
        // mapping item whose first key sits on the dash line
        Json obj = Json::object();
        add_entry(obj, rest, item_col);
        while (pos_ < lines_.size() && lines_[pos_].indent == item_col && !is_seq_item(lines_[pos_].text)) {
          std::string t = lines_[pos_].text;
          ++pos_;
          add_entry(obj, t, item_col);
        }
        arr.push_back(obj);
      } else {
        arr.push_back(scalar(rest));
      }
    }
    return arr;
  }

  void add_entry(Json& obj, const std::string& text, int indent) {
    size_t c = key_colon(text);
    if (c == std::string::npos) throw JsonError("yaml: expected 'key: value' in '" + text + "'");
    std::string key = unquote_key(text.substr(0, c));
    std::string val = trim(text.substr(c + 1));
    if (!val.empty()) {
      obj[key] = scalar(val);
      return;
    }
    // nested block: deeper indent, or a sequence at the same indent
    if (pos_ < lines_.size() &&
        (lines_[pos_].indent > indent || (lines_[pos_].indent == indent && is_seq_item(lines_[pos_].text)))) {
      obj[key] = parse_block(lines_[pos_].indent);
    } else {
      obj[key] = Json();
    }
  }

  Json parse_map(int indent) {
    Json obj = Json::object();
    while (pos_ < lines_.size() && lines_[pos_].indent == indent && !is_seq_item(lines_[pos_].text)) {
      std::string t = lines_[pos_].text;
      ++pos_;
      add_entry(obj, t, indent);
    }
    return obj;
  }

  std::vector<Line> lines_;
  size_t pos_ = 0;
};

}  // namespace

Json yaml_parse(const std::string& text) {
  std::vector<Line> lines;
  size_t start = 0;
  while (start <= text.size()) {
    size_t nl = text.find('\n', start);
    std::string raw = text.substr(start, nl == std::string::npos ? std::string::npos : nl - start);
    start = nl == std::string::npos ? text.size() + 1 : nl + 1;
    std::string body = rtrim(strip_comment(raw));
    if (trim(body).empty() || trim(body) == "---") continue;
    int ind = 0;
    while (ind < (int)body.size() && body[ind] == ' ') ++ind;
    lines.push_back({ind, body.substr(ind)});
  }
  YamlParser p(std::move(lines));
  return p.parse_document();
}

std::string render_template(const std::string& tmpl,
                            const std::vector<std::pair<std::string, std::string>>& values) {
  std::string out;
  size_t i = 0;
  while (i < tmpl.size()) {
    size_t a = tmpl.find("{{", i);
    if (a == std::string::npos) {
      out += tmpl.substr(i);
      break;
    }
    size_t b = tmpl.find("}}", a);
    if (b == std::string::npos) throw JsonError("template: unterminated action");
    out += tmpl.substr(i, a - i);
    std::string key = trim(tmpl.substr(a + 2, b - a - 2));
    if (!key.empty() && key[0] == '.') key = key.substr(1);
    bool found = false;
    for (const auto& kv : values) {
      if (kv.first == key) {
        out += kv.second;
        found = true;
        break;
      }
    }
    if (!found) throw JsonError("template: unknown field ." + key);
    i = b + 2;
  }
  return out;
}

}  // namespace pto
