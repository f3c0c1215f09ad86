// Hand-written recursive-descent TCAP parser (the reference uses flex/bison: Lexer.l / Parser.y).
//   <tupleSpec> <= APPLY (<in>, <proj>, 'comp', 'lambda')
//   <tupleSpec> <= FILTER (<in>, <proj>, 'comp')
//   <tupleSpec> <= HASHLEFT|HASHRIGHT (<in>, <proj>, 'comp', 'lambda')
//   <tupleSpec> <= HASHONE|FLATTEN (<in>, <proj>, 'comp')
//   <tupleSpec> <= JOIN (<in1>, <proj1>, <in2>, <proj2>, 'comp')
//   <tupleSpec> <= AGGREGATE|PARTITION (<in>, 'comp')
//   <tupleSpec> <= SCAN ('db', 'set', 'comp')
//   <tupleSpec> <= OUTPUT (<in>, 'db', 'set', 'comp')
// Keywords are case-insensitive; /* */ and # / // comments are skipped.
#include <cctype>
#include <stdexcept>

#include "runtime.h"

namespace nsdb_rt {
namespace {

enum Tok { T_ID, T_STR, T_LP, T_RP, T_COMMA, T_GETS, T_EOF };

struct Lexer {
  const std::string& s;
  size_t i = 0;
  int line = 1;
  explicit Lexer(const std::string& src) : s(src) {}

  void skip() {
    for (;;) {
      while (i < s.size() && std::isspace((unsigned char)s[i])) {
        if (s[i] == '\n') ++line;
        ++i;
      }
      if (i + 1 < s.size() && s[i] == '/' && s[i + 1] == '*') {
        size_t e = s.find("*/", i + 2);
        for (size_t k = i; k < (e == std::string::npos ? s.size() : e); ++k)
          if (s[k] == '\n') ++line;
        i = (e == std::string::npos) ? s.size() : e + 2;
        continue;
      }
      if (i < s.size() && (s[i] == '#' || (s[i] == '/' && i + 1 < s.size() && s[i + 1] == '/'))) {
        while (i < s.size() && s[i] != '\n') ++i;
        continue;
      }
      break;
    }
  }

  Tok next(std::string& text) {
    skip();
    if (i >= s.size()) return T_EOF;
    char c = s[i];
    if (c == '(') { ++i; return T_LP; }
    if (c == ')') { ++i; return T_RP; }
    if (c == ',') { ++i; return T_COMMA; }
    if (c == '<' && i + 1 < s.size() && s[i + 1] == '=') { i += 2; return T_GETS; }
    if (c == '\'' || c == '"') {
      size_t e = s.find(c, i + 1);
      if (e == std::string::npos) throw std::runtime_error("TCAP line " + std::to_string(line) + ": unterminated string");
      text = s.substr(i + 1, e - i - 1);
      i = e + 1;
      return T_STR;
    }
    if (std::isalnum((unsigned char)c) || c == '_' || c == '-' || c == '=' || c == '&' || c == '|' || c == '.') {
      size_t b = i;
      while (i < s.size() && (std::isalnum((unsigned char)s[i]) || s[i] == '_' || s[i] == '-' || s[i] == '=' ||
                              s[i] == '&' || s[i] == '|' || s[i] == '.'))
        ++i;
      text = s.substr(b, i - b);
      return T_ID;
    }
    throw std::runtime_error("TCAP line " + std::to_string(line) + ": unexpected character '" + std::string(1, c) + "'");
  }
};

struct Parser {
  Lexer lx;
  Tok tok;
  std::string text;
  explicit Parser(const std::string& s) : lx(s) { advance(); }
  void advance() { tok = lx.next(text); }
  [[noreturn]] void fail(const std::string& what) {
    throw std::runtime_error("TCAP parse error at line " + std::to_string(lx.line) + ": " + what);
  }
  void expect(Tok t, const char* what) {
    if (tok != t) fail(std::string("expected ") + what);
    advance();
  }
  std::string ident() {
    if (tok != T_ID) fail("expected identifier");
    std::string r = text;
    advance();
    return r;
  }
  std::string str() {
    if (tok != T_STR) fail("expected quoted string");
    std::string r = text;
    advance();
    return r;
  }
  TupleSpec spec() {
    TupleSpec t;
    t.name = ident();
    expect(T_LP, "'('");
    if (tok != T_RP) {
      t.atts.push_back(ident());
      while (tok == T_COMMA) {
        advance();
        t.atts.push_back(ident());
      }
    }
    expect(T_RP, "')'");
    return t;
  }
  static std::string upper(std::string s) {
    for (auto& c : s) c = (char)std::toupper((unsigned char)c);
    return s;
  }

  AtomicComputation atom() {
    AtomicComputation a;
    a.line = lx.line;
    a.output = spec();
    expect(T_GETS, "'<='");
    a.type = upper(ident());
    if (a.type == "AGG") a.type = "AGGREGATE";
    expect(T_LP, "'('");
    if (a.type == "APPLY" || a.type == "HASHLEFT" || a.type == "HASHRIGHT") {
      a.input = spec(); expect(T_COMMA, "','");
      a.projection = spec(); expect(T_COMMA, "','");
      a.comp = str(); expect(T_COMMA, "','");
      a.lambda = str();
    } else if (a.type == "FILTER" || a.type == "HASHONE" || a.type == "FLATTEN") {
      a.input = spec(); expect(T_COMMA, "','");
      a.projection = spec(); expect(T_COMMA, "','");
      a.comp = str();
    } else if (a.type == "JOIN") {
      a.input = spec(); expect(T_COMMA, "','");
      a.projection = spec(); expect(T_COMMA, "','");
      a.input2 = spec(); expect(T_COMMA, "','");
      a.projection2 = spec(); expect(T_COMMA, "','");
      a.comp = str();
    } else if (a.type == "AGGREGATE" || a.type == "PARTITION") {
      a.input = spec(); expect(T_COMMA, "','");
      a.comp = str();
    } else if (a.type == "SCAN") {
      a.db = str(); expect(T_COMMA, "','");
      a.set = str(); expect(T_COMMA, "','");
      a.comp = str();
    } else if (a.type == "OUTPUT") {
      a.input = spec(); expect(T_COMMA, "','");
      a.db = str(); expect(T_COMMA, "','");
      a.set = str(); expect(T_COMMA, "','");
      a.comp = str();
    } else {
      fail("unknown atomic computation '" + a.type + "'");
    }
    expect(T_RP, "')'");
    return a;
  }

  std::vector<AtomicComputation> all() {
    std::vector<AtomicComputation> out;
    while (tok != T_EOF) out.push_back(atom());
    return out;
  }
};

}  // namespace

std::vector<AtomicComputation> parse_tcap(const std::string& text) {
  Parser p(text);
  auto atoms = p.all();
  // semantic check: every consumed tuple set must be produced earlier (or be produced by SCAN)
  std::unordered_map<std::string, const AtomicComputation*> produced;
  for (const auto& a : atoms) {
    auto need = [&](const TupleSpec& t) {
      if (t.name.empty()) return;
      auto it = produced.find(t.name);
      if (it == produced.end())
        throw std::runtime_error("TCAP line " + std::to_string(a.line) + ": tuple set '" + t.name + "' used before definition");
      for (const auto& att : t.atts) {
        bool found = false;
        for (const auto& o : it->second->output.atts) found |= (o == att);
        if (!found)
          throw std::runtime_error("TCAP line " + std::to_string(a.line) + ": attribute '" + att + "' not in '" + t.name + "'");
      }
    };
    need(a.input); need(a.projection); need(a.input2); need(a.projection2);
    if (produced.count(a.output.name))
      throw std::runtime_error("TCAP line " + std::to_string(a.line) + ": tuple set '" + a.output.name + "' redefined");
    produced[a.output.name] = &a;
  }
  return atoms;
}

}  // namespace nsdb_rt
