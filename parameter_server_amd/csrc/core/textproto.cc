#include "textproto.h"

#include <cctype>
#include <sstream>

namespace pscore {

namespace {

class Lexer {
 public:
  explicit Lexer(const std::string& s) : s_(s) {}

  [[noreturn]] void fail(const std::string& what) const {
    std::ostringstream os;
    os << "textproto:" << line_ << ":" << col_ << ": " << what;
    throw TextProtoError(os.str());
  }

  void skip_ws() {
    while (pos_ < s_.size()) {
      const char c = s_[pos_];
      if (c == '#') {
        while (pos_ < s_.size() && s_[pos_] != '\n') adv();
      } else if (std::isspace((unsigned char)c)) {
        adv();
      } else {
        break;
      }
    }
  }

  bool eof() {
    skip_ws();
    return pos_ >= s_.size();
  }

  char peek() {
    skip_ws();
    return pos_ < s_.size() ? s_[pos_] : '\0';
  }

  bool accept(char c) {
    if (peek() == c) {
      adv();
      return true;
    }
    return false;
  }

  void expect(char c) {
    if (!accept(c)) fail(std::string("expected '") + c + "'");
  }

  std::string ident() {
    skip_ws();
    const size_t b = pos_;
    while (pos_ < s_.size() && (std::isalnum((unsigned char)s_[pos_]) || s_[pos_] == '_' ||
                                s_[pos_] == '.'))
      adv();
    if (b == pos_) fail("expected identifier");
    return s_.substr(b, pos_ - b);
  }

  // field name: identifier or [extension.name]
  std::string field_name() {
    if (accept('[')) {
      std::string n = ident();
      expect(']');
      return "[" + n + "]";
    }
    return ident();
  }

  TPValue scalar() {
    skip_ws();
    TPValue v;
    const char c = peek();
    if (c == '"' || c == '\'') {
      v.kind = TPValue::kString;
      while (peek() == '"' || peek() == '\'') v.text += quoted();
      return v;
    }
    const size_t b = pos_;
    if (c == '-' || c == '+') adv();
    while (pos_ < s_.size() && (std::isalnum((unsigned char)s_[pos_]) || s_[pos_] == '.' ||
                                s_[pos_] == '_' ||
                                ((s_[pos_] == '-' || s_[pos_] == '+') && pos_ > b &&
                                 (s_[pos_ - 1] == 'e' || s_[pos_ - 1] == 'E'))))
      adv();
    if (b == pos_) fail("expected value");
    v.text = s_.substr(b, pos_ - b);
    const char f = v.text[0];
    const bool numeric = std::isdigit((unsigned char)f) || f == '.' ||
                         ((f == '-' || f == '+') && v.text.size() > 1);
    v.kind = numeric ? TPValue::kNumber : TPValue::kIdent;
    return v;
  }

 private:
  void adv() {
    if (s_[pos_] == '\n') {
      ++line_;
      col_ = 1;
    } else {
      ++col_;
    }
    ++pos_;
  }

  std::string quoted() {
    const char q = s_[pos_];
    adv();
    std::string out;
    while (true) {
      if (pos_ >= s_.size() || s_[pos_] == '\n') fail("unterminated string");
      char c = s_[pos_];
      adv();
      if (c == q) break;
      if (c == '\\') {
        if (pos_ >= s_.size()) fail("bad escape");
        char e = s_[pos_];
        adv();
        switch (e) {
          case 'n': out += '\n'; break;
          case 't': out += '\t'; break;
          case 'r': out += '\r'; break;
          case '\\': out += '\\'; break;
          case '\'': out += '\''; break;
          case '"': out += '"'; break;
          case 'x': {
            int v = 0, k = 0;
            while (k < 2 && pos_ < s_.size() && std::isxdigit((unsigned char)s_[pos_])) {
              v = v * 16 + (std::isdigit((unsigned char)s_[pos_]) ? s_[pos_] - '0'
                                                                   : (std::tolower(s_[pos_]) - 'a' + 10));
              adv();
              ++k;
            }
            out += (char)v;
            break;
          }
          default:
            if (e >= '0' && e <= '7') {
              int v = e - '0', k = 1;
              while (k < 3 && pos_ < s_.size() && s_[pos_] >= '0' && s_[pos_] <= '7') {
                v = v * 8 + (s_[pos_] - '0');
                adv();
                ++k;
              }
              out += (char)v;
            } else {
              out += e;
            }
        }
      } else {
        out += c;
      }
    }
    return out;
  }

  const std::string& s_;
  size_t pos_ = 0;
  int line_ = 1, col_ = 1;
};

std::shared_ptr<TPMessage> parse_body(Lexer& lx, char close) {
  auto m = std::make_shared<TPMessage>();
  while (true) {
    if (close == '\0') {
      if (lx.eof()) break;
    } else if (lx.accept(close)) {
      break;
    } else if (lx.eof()) {
      lx.fail(std::string("missing '") + close + "'");
    }
    std::string name = lx.field_name();
    TPValue v;
    const bool colon = lx.accept(':');
    const char c = lx.peek();
    if (c == '{' || c == '<') {
      lx.accept(c);
      v.kind = TPValue::kMessage;
      v.msg = parse_body(lx, c == '{' ? '}' : '>');
    } else if (c == '[' && colon) {  // list syntax: f: [a, b, c]
      lx.accept('[');
      if (!lx.accept(']')) {
        while (true) {
          TPValue e = lx.peek() == '{' ? TPValue{} : lx.scalar();
          if (lx.peek() == '{') {
            lx.accept('{');
            e.kind = TPValue::kMessage;
            e.msg = parse_body(lx, '}');
          }
          m->fields.emplace_back(name, e);
          if (lx.accept(']')) break;
          lx.expect(',');
        }
      }
      lx.accept(',') || lx.accept(';');
      continue;
    } else {
      if (!colon) lx.fail("expected ':' after field '" + name + "'");
      v = lx.scalar();
    }
    m->fields.emplace_back(name, v);
    lx.accept(',') || lx.accept(';');
  }
  return m;
}

}  // namespace

TPMessage parse_textproto(const std::string& src) {
  Lexer lx(src);
  return *parse_body(lx, '\0');
}

std::string escape_string(const std::string& s) {
  std::string o = "\"";
  for (char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\t': o += "\\t"; break;
      default: o += c;
    }
  }
  return o + "\"";
}

std::string print_textproto(const TPMessage& m, int indent) {
  std::ostringstream os;
  const std::string pad(indent * 2, ' ');
  for (const auto& [name, v] : m.fields) {
    if (v.kind == TPValue::kMessage) {
      os << pad << name << " {\n" << print_textproto(*v.msg, indent + 1) << pad << "}\n";
    } else if (v.kind == TPValue::kString) {
      os << pad << name << ": " << escape_string(v.text) << "\n";
    } else {
      os << pad << name << ": " << v.text << "\n";
    }
  }
  return os.str();
}

}  // namespace pscore
