#include "filter.h"

#include <stdexcept>

namespace tpi {

namespace {

// Expand '{a,b}' groups (rclone forbids nesting) into plain alternatives.
std::vector<std::string> expand_braces(const std::string& g) {
  std::vector<std::string> out{""};
  size_t i = 0;
  while (i < g.size()) {
    char c = g[i];
    if (c == '\\' && i + 1 < g.size()) {
      for (auto& s : out) s += g.substr(i, 2);
      i += 2;
      continue;
    }
    if (c == '[') {  // copy a class verbatim (may contain '{' or ',')
      size_t j = i + 1;
      if (j < g.size() && (g[j] == '^' || g[j] == '!')) ++j;
      if (j < g.size() && g[j] == ']') ++j;
      while (j < g.size() && g[j] != ']') j += (g[j] == '\\') ? 2 : 1;
      if (j >= g.size()) throw std::invalid_argument("mismatched '[' and ']' in glob " + g);
      for (auto& s : out) s += g.substr(i, j - i + 1);
      i = j + 1;
      continue;
    }
    if (c == '{') {
      size_t j = g.find('}', i);
      if (j == std::string::npos) throw std::invalid_argument("mismatched '{' and '}' in glob " + g);
      std::string body = g.substr(i + 1, j - i - 1);
      if (body.find('{') != std::string::npos)
        throw std::invalid_argument("can't nest '{' '}' in glob " + g);
      std::vector<std::string> parts;
      size_t s = 0;
      for (size_t k = 0; k <= body.size(); ++k)
        if (k == body.size() || body[k] == ',') {
          parts.push_back(body.substr(s, k - s));
          s = k + 1;
        }
      std::vector<std::string> next;
      for (auto& o : out)
        for (auto& p : parts) next.push_back(o + p);
      out.swap(next);
      i = j + 1;
      continue;
    }
    if (c == '}') throw std::invalid_argument("mismatched '{' and '}' in glob " + g);
    for (auto& s : out) s += c;
    ++i;
  }
  return out;
}

std::vector<GlobTok> tokenize(const std::string& g) {
  std::vector<GlobTok> toks;
  for (size_t i = 0; i < g.size();) {
    char c = g[i];
    GlobTok t;
    if (c == '\\' && i + 1 < g.size()) {
      t.kind = GlobTok::LIT;
      t.lit = g[i + 1];
      i += 2;
    } else if (c == '*') {
      size_t n = 0;
      while (i < g.size() && g[i] == '*') ++n, ++i;
      if (n > 2) throw std::invalid_argument("too many stars in glob " + g);
      t.kind = n == 2 ? GlobTok::DSTAR : GlobTok::STAR;
    } else if (c == '?') {
      t.kind = GlobTok::QMARK;
      ++i;
    } else if (c == '[') {
      t.kind = GlobTok::CLASS;
      size_t j = i + 1;
      if (j < g.size() && g[j] == '^') t.neg = true, ++j;
      bool first = true;
      while (j < g.size() && (g[j] != ']' || first)) {
        unsigned char lo = (unsigned char)g[j];
        if (lo == '\\' && j + 1 < g.size()) lo = (unsigned char)g[++j];
        unsigned char hi = lo;
        if (j + 2 < g.size() && g[j + 1] == '-' && g[j + 2] != ']') {
          hi = (unsigned char)g[j + 2];
          j += 2;
        }
        t.ranges.emplace_back(lo, hi);
        ++j;
        first = false;
      }
      if (j >= g.size()) throw std::invalid_argument("mismatched '[' and ']' in glob " + g);
      i = j + 1;
    } else if (c == ']') {
      throw std::invalid_argument("mismatched ']' in glob " + g);
    } else {
      t.kind = GlobTok::LIT;
      t.lit = c;
      ++i;
    }
    toks.push_back(std::move(t));
  }
  return toks;
}

bool class_match(const GlobTok& t, unsigned char c) {
  bool in = false;
  for (auto& r : t.ranges)
    if (c >= r.first && c <= r.second) {
      in = true;
      break;
    }
  return in != t.neg;
}

bool match_at(const std::vector<GlobTok>& toks, size_t ti, const std::string& s, size_t si) {
  while (ti < toks.size()) {
    const GlobTok& t = toks[ti];
    switch (t.kind) {
      case GlobTok::LIT:
        if (si >= s.size() || s[si] != t.lit) return false;
        ++si, ++ti;
        break;
      case GlobTok::QMARK:
        if (si >= s.size() || s[si] == '/') return false;
        ++si, ++ti;
        break;
      case GlobTok::CLASS:
        if (si >= s.size() || !class_match(t, (unsigned char)s[si])) return false;
        ++si, ++ti;
        break;
      case GlobTok::STAR:
        for (size_t k = si;; ++k) {
          if (match_at(toks, ti + 1, s, k)) return true;
          if (k >= s.size() || s[k] == '/') return false;
        }
      case GlobTok::DSTAR:
        for (size_t k = si; k <= s.size(); ++k)
          if (match_at(toks, ti + 1, s, k)) return true;
        return false;
    }
  }
  return si == s.size();
}

}  // namespace

Glob::Glob(const std::string& glob) : source_(glob) {
  std::string g = glob;
  if (!g.empty() && g[0] == '/') {
    anchored_ = true;
    g = g.substr(1);
  }
  for (auto& alt : expand_braces(g)) alts_.push_back(tokenize(alt));
}

bool Glob::match(const std::string& path) const {
  for (auto& toks : alts_) {
    if (match_at(toks, 0, path, 0)) return true;
    if (!anchored_)
      for (size_t i = 0; i < path.size(); ++i)
        if (path[i] == '/' && match_at(toks, 0, path, i + 1)) return true;
  }
  return false;
}

void Filter::add_rule(const std::string& rule) {
  if (rule.size() >= 2 && (rule[0] == '+' || rule[0] == '-') && rule[1] == ' ') {
    add(rule[0] == '+', rule.substr(2));
    return;
  }
  throw std::invalid_argument("malformed rule " + rule);
}

void Filter::add(bool include, const std::string& glob_in) {
  std::string glob = glob_in;
  bool dir_rule = !glob.empty() && glob.back() == '/';
  bool file_rule = !dir_rule;
  if (dir_rule && !include) glob += "**";  // excluding "dir/" == excluding "dir/**"
  if (glob.find("**") != std::string::npos) dir_rule = file_rule = true;
  if (file_rule) {
    file_rules_.push_back({include, Glob(glob)});
    if (include || glob == "*") {
      // Directories that may lead to an included file must be traversed.
      for (size_t i = glob.size(); i-- > 0;) {
        if (glob[i] != '/') continue;
        std::string prefix = glob.substr(0, i + 1);
        if (prefix == "/") continue;
        dir_rules_.push_back({include, Glob(prefix)});
      }
    }
  }
  if (dir_rule) dir_rules_.push_back({include, Glob(glob)});
}

bool Filter::eval(const std::vector<Rule>& rules, const std::string& path) {
  for (auto& r : rules)
    if (r.glob.match(path)) return r.include;
  return true;
}

bool Filter::include_file(const std::string& rel) const { return eval(file_rules_, rel); }

bool Filter::include_dir(const std::string& rel) const {
  if (rel.empty()) return true;
  return eval(dir_rules_, rel + "/");
}

std::vector<std::string> Filter::describe() const {
  std::vector<std::string> out;
  for (auto& r : file_rules_) out.push_back(std::string("file ") + (r.include ? "+ " : "- ") + r.glob.source());
  for (auto& r : dir_rules_) out.push_back(std::string("dir ") + (r.include ? "+ " : "- ") + r.glob.source());
  return out;
}

}  // namespace tpi
