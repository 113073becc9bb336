// Minimal protobuf *text format* parser/printer (no protobuf runtime on the box).
//
// The reference ships its whole app configuration as text-format protos
// (AppConfig / LM.Config, src/app/main/proto/app.proto, linear.proto), read by
// the scheduler from --app_file/--app_conf and broadcast to every node
// (src/system/postoffice.cc:61-70). This parser accepts that syntax:
//   field: scalar | field { ... } | field: { ... } | field < ... >
//   [ext.field.name]: scalar        (proto2 extensions, e.g. [PS.LM.delta_init_value])
//   "double" / 'single' quoted strings with C escapes, adjacent-string concat
//   numbers (1, -2, .01, 2e-5, 0x1F, inf/nan), identifiers (enums, true/false)
//   '#' comments, optional ',' / ';' separators
// into an ordered tree; schema mapping (types, defaults) happens in Python.
#pragma once
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace pscore {

struct TPMessage;

struct TPValue {
  enum Kind { kNumber, kIdent, kString, kMessage };
  Kind kind = kIdent;
  std::string text;                 // scalar text (unescaped for strings)
  std::shared_ptr<TPMessage> msg;   // for kMessage
};

struct TPMessage {
  std::vector<std::pair<std::string, TPValue>> fields;  // in source order (repeated = repeated names)
};

class TextProtoError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

TPMessage parse_textproto(const std::string& src);
std::string print_textproto(const TPMessage& m, int indent = 0);
std::string escape_string(const std::string& s);

}  // namespace pscore
