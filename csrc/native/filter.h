// rclone-compatible include/exclude filter rules (the semantics the reference gets from
// rclone's fs/filter package via task/common/machine/storage.go:123-159,267-280).
//
// Glob language: leading '/' anchors at the transfer root, otherwise a pattern matches at
// any directory level; '*' = any run of non-'/' characters, '**' = anything, '?' = one
// non-'/' character, '[...]' character classes, '{a,b}' alternatives, '\' escapes.
// Rules are evaluated in order and the first match decides; no match = include.
// Directory rules are matched against "dir/" and decide whether a directory is traversed
// (and created, empty or not), exactly like rclone's dirRules.
#pragma once
#include <string>
#include <vector>

namespace tpi {

struct GlobTok {
  enum Kind { LIT, STAR, DSTAR, QMARK, CLASS } kind;
  char lit = 0;
  bool neg = false;
  std::vector<std::pair<unsigned char, unsigned char>> ranges;
};

class Glob {
 public:
  explicit Glob(const std::string& glob);  // throws std::invalid_argument
  bool match(const std::string& path) const;
  const std::string& source() const { return source_; }

 private:
  std::string source_;
  bool anchored_ = false;
  std::vector<std::vector<GlobTok>> alts_;  // brace alternatives expanded
};

class Filter {
 public:
  // rule: "+ glob" or "- glob" (rclone filter-rule syntax).
  void add_rule(const std::string& rule);
  void add(bool include, const std::string& glob);
  bool include_file(const std::string& rel) const;  // rel: "a/b.txt" (no leading '/')
  bool include_dir(const std::string& rel) const;   // rel: "a/b"
  std::vector<std::string> describe() const;

 private:
  struct Rule {
    bool include;
    Glob glob;
  };
  static bool eval(const std::vector<Rule>& rules, const std::string& path);
  std::vector<Rule> file_rules_, dir_rules_;
};

}  // namespace tpi
