// scene_dsl.cpp -- host front end for the reference's scene DSL.
//
// Restates src/sceneparser: the PEG grammar (scene_grammar.pest:1-74, including its implicit
// WHITESPACE = " " | "\n" | "\r" | comment -- no tab), the AST lowering (ast_node.rs:267-736,
// keeping only the FIRST operator of an `a op b op c` chain, :598-629) and the tree-walking
// evaluator (ast_node.rs:150-265, 438-596; context.rs) with its globals / call-frame locals.
// Objects are lowered to rt_shape_* / rt_scene_add_object calls exactly where the reference
// calls Shape::to_rt_object + RayTracer::add_object (ast_node.rs:176-191).
#include <stdlib.h>
#include <string.h>

#include <array>
#include <map>
#include <mutex>
#include <stdexcept>
#include <memory>
#include <string>
#include <vector>

#include "scene.h"

namespace rt {
namespace {

// Decoded textures, process-wide, keyed by the PNG file's bytes (a 64-bit FNV-1a and the size, then the
// bytes compared in full): a hit is the same file content, so the same pixels.  At most 8 images are
// kept (least recently used dropped).
struct DecodedPng {
  std::vector<uint8_t> file;
  std::vector<uint8_t> rgba;
  uint32_t w = 0, h = 0;
  uint64_t last_use = 0;
};
std::shared_ptr<const DecodedPng> decoded_png(const std::vector<uint8_t>& file) {
  static std::mutex mu;
  static std::map<std::pair<uint64_t, size_t>, std::shared_ptr<DecodedPng>> cache;
  static uint64_t clock = 0;
  uint64_t hsh = 1469598103934665603ull;
  for (uint8_t b : file) hsh = (hsh ^ b) * 1099511628211ull;
  const auto key = std::make_pair(hsh, file.size());
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end() && it->second->file == file) {
      it->second->last_use = ++clock;
      return it->second;
    }
  }
  auto img = std::make_shared<DecodedPng>();
  if (png_decode_rgba8(file, &img->rgba, &img->w, &img->h)) return nullptr;
  img->file = file;
  std::lock_guard<std::mutex> lk(mu);
  img->last_use = ++clock;
  if (cache.size() >= 8 && !cache.count(key)) {
    auto lru = cache.begin();
    for (auto it = cache.begin(); it != cache.end(); ++it)
      if (it->second->last_use < lru->second->last_use) lru = it;
    cache.erase(lru);
  }
  cache[key] = img;
  return img;
}

// ------------------------------------------------------------------ values (value.rs:5-14)
struct DslShape;
struct Value {
  enum Kind { NONE, NUMBER, BOOLEAN, STRING, COLOR, VECTOR, OBJECT, TEXTURE } kind = NONE;
  double num = 0.0;
  bool boolean = false;
  std::string str;
  double c[4] = {0, 0, 0, 0};     // Value::Color {r,g,b,a}
  double v[3] = {0, 0, 0};        // Value::Vector
  std::shared_ptr<const DslShape> shape;
  int32_t texture = -1;
};

// sceneparser/shape.rs:7-35
struct DslShape {
  enum Kind { SPHERE, CUBE, PLANE, CSG } kind;
  bool textured = false;
  double color[4] = {0, 0, 0, 1};
  int32_t texture = -1;
  double reflectivity = 0, transparency = 0;
  double center[3] = {0, 0, 0};
  double size = 1.0;              // radius / length
  double normal[3] = {0, 1, 0};
  double distance = 1.0;
  rt_csg_op op = RT_CSG_UNION;
  std::shared_ptr<const DslShape> a, b;
  rt_transformation t;
};

// ------------------------------------------------------------------ AST (ast_node.rs:35-81)
struct Expr;
using ExprP = std::unique_ptr<Expr>;
struct Expr {
  enum Kind { VALUE, REF, VECTOR, RGB, OBJECT, TEXTURE, MINUS, BINOP } kind;
  Value value;
  std::string id;                  // REF name / OBJECT shape name
  ExprP x, y, z;                   // parts, binop operands (x, y), minus/texture operand (x)
  char op = 0;                     // + - * / % < >
  std::vector<ExprP> params;
};
struct Stmt;
using StmtP = std::shared_ptr<Stmt>;
struct Stmt {
  enum Kind { LIST, ASSIGN, FUNCTION, CALL, DRAW, XFORM, IF, WHILE, LIGHT, CAMERA } kind;
  std::vector<StmtP> list;
  bool local = false;
  std::string id;                  // assign target / function / call name / command
  ExprP expr;
  std::vector<ExprP> params;
  std::vector<std::string> names;  // function parameters
  StmtP body;
  ExprP x, y, z;
  char xform = 0;                  // 't' 'r' 's'
};

// ------------------------------------------------------------------ PEG parser
class Parser {
 public:
  Parser(const char* s) : s_(s), n_(strlen(s)) {}
  size_t pos = 0, furthest = 0;
  std::string unimplemented;       // "display" / "append" command (ast_node.rs:354 panics)

  bool eof() const { return pos >= n_; }
  char at(size_t k = 0) const { return pos + k < n_ ? s_[pos + k] : '\0'; }
  void mark() { if (pos > furthest) furthest = pos; }

  static bool alpha(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }
  static bool digit(char c) { return c >= '0' && c <= '9'; }
  static bool alnum(char c) { return alpha(c) || digit(c) || c == '_'; }

  // one WHITESPACE token (pest:2-3)
  bool ws1() {
    char c = at();
    if (c == ' ' || c == '\n' || c == '\r') { ++pos; return true; }
    if (c == '/' && at(1) == '/') {
      pos += 2;
      while (!eof() && s_[pos] != '\n') ++pos;
      if (!eof()) ++pos;
      return true;
    }
    return false;
  }
  void ws() { while (ws1()) {} }
  bool lit(const char* l) {
    size_t k = strlen(l);
    if (pos + k <= n_ && memcmp(s_ + pos, l, k) == 0) { pos += k; return true; }
    mark();
    return false;
  }
  bool kw(const char* k) {            // @{ "k" ~ !alnum }
    size_t save = pos;
    if (!lit(k)) return false;
    if (alnum(at())) { pos = save; mark(); return false; }
    return true;
  }
  const char* kw_any(std::initializer_list<const char*> ks) {
    for (const char* k : ks) if (kw(k)) return k;
    return nullptr;
  }
  bool keyword_ahead() {              // keyword (pest:50)
    size_t save = pos;
    bool r = kw("local") || kw_any({"scale", "rotate", "translate"}) ||
             kw_any({"draw", "display", "append"}) || kw_any({"sphere", "plane", "csg", "cube"}) ||
             kw("function");
    pos = save;
    return r;
  }
  bool id(std::string* out) {         // id = @{ !keyword ~ ident } (pest:9,51)
    if (keyword_ahead()) { mark(); return false; }
    char c = at();
    if (!(alpha(c) || c == '_')) { mark(); return false; }
    size_t st = pos;
    while (alnum(at())) ++pos;
    out->assign(s_ + st, pos - st);
    return true;
  }

  // param_list = { (expression ~ ","?)* } (pest:30)
  std::vector<ExprP> param_list() {
    std::vector<ExprP> out;
    for (;;) {
      size_t save = pos;
      if (!out.empty()) ws();
      ExprP e = expression();
      if (!e) { pos = save; break; }
      out.push_back(std::move(e));
      size_t s2 = pos;
      ws();
      if (!lit(",")) pos = s2;
    }
    return out;
  }

  ExprP number() {                    // @{ digit+ ~ ("." ~ digit+)? ~ !alpha } (pest:53)
    size_t st = pos;
    if (!digit(at())) { mark(); return nullptr; }
    while (digit(at())) ++pos;
    if (at() == '.' && digit(at(1))) { ++pos; while (digit(at())) ++pos; }
    if (alpha(at())) { pos = st; mark(); return nullptr; }
    std::string lexeme(s_ + st, pos - st);
    ExprP e(new Expr{Expr::VALUE});
    e->value.kind = Value::NUMBER;
    e->value.num = strtod(lexeme.c_str(), nullptr);   // str::parse::<f64>: correctly rounded
    return e;
  }
  ExprP string_lit() {                // pest:54
    char q = at();
    if (q != '"' && q != '\'') { mark(); return nullptr; }
    size_t e = pos + 1;
    while (e < n_ && s_[e] != q) ++e;
    if (e >= n_) { mark(); return nullptr; }
    ExprP x(new Expr{Expr::VALUE});
    x->value.kind = Value::STRING;
    x->value.str.assign(s_ + pos + 1, e - pos - 1);
    pos = e + 1;
    return x;
  }
  // value (pest:71-74), ordered choice with backtracking
  ExprP value() {
    size_t save = pos;
    if (ExprP e = number()) return e;
    pos = save;
    if (const char* c = kw_any({"red", "orange", "yellow", "green", "blue", "purple", "black", "white"})) {
      static const std::map<std::string, std::vector<double>> cols = {       // ast_node.rs:661-675
          {"red", {1, 0, 0}}, {"orange", {1, 0.5, 0}}, {"yellow", {1, 1, 0}}, {"green", {0, 1, 0}},
          {"blue", {0, 0, 1}}, {"purple", {1, 0, 1}}, {"black", {0, 0, 0}}, {"white", {1, 1, 1}}};
      const std::vector<double>& k = cols.at(c);
      ExprP e(new Expr{Expr::VALUE});
      e->value.kind = Value::COLOR;
      e->value.c[0] = k[0]; e->value.c[1] = k[1]; e->value.c[2] = k[2]; e->value.c[3] = 1.0;
      return e;
    }
    pos = save;
    if (lit("rgb")) {                 // color = { "rgb" ~ "(" ~ (expression ~ ","?){3} ~ ")" }
      ws();
      if (lit("(")) {
        ExprP parts[3];
        bool ok = true;
        for (int i = 0; i < 3 && ok; ++i) {
          ws();
          parts[i] = expression();
          if (!parts[i]) { ok = false; break; }
          size_t s2 = pos; ws(); if (!lit(",")) pos = s2;
        }
        if (ok) {
          ws();
          if (lit(")")) {
            ExprP e(new Expr{Expr::RGB});
            e->x = std::move(parts[0]); e->y = std::move(parts[1]); e->z = std::move(parts[2]);
            return e;
          }
        }
      }
    }
    pos = save;
    if (lit("<")) {                   // vector = { "<" ~ e ~ "," ~ e ~ "," ~ e ~ ">" }
      ExprP p[3];
      bool ok = true;
      for (int i = 0; i < 3 && ok; ++i) {
        ws();
        p[i] = expression();
        if (!p[i]) { ok = false; break; }
        ws();
        if (!lit(i < 2 ? "," : ">")) ok = false;
      }
      if (ok) {
        ExprP e(new Expr{Expr::VECTOR});
        e->x = std::move(p[0]); e->y = std::move(p[1]); e->z = std::move(p[2]);
        return e;
      }
    }
    pos = save;
    if (lit("texture")) {             // texture = { "texture" ~ "(" ~ expression ~ ")" }
      ws();
      if (lit("(")) {
        ws();
        ExprP x = expression();
        if (x) { ws(); if (lit(")")) { ExprP e(new Expr{Expr::TEXTURE}); e->x = std::move(x); return e; } }
      }
    }
    pos = save;
    if (lit("(")) {                   // "(" ~ expression ~ ")"
      ws();
      ExprP x = expression();
      if (x) { ws(); if (lit(")")) return x; }
    }
    pos = save;
    if (const char* name = kw_any({"sphere", "plane", "csg", "cube"})) {   // object
      ws();
      if (lit("(")) {
        ws();
        std::vector<ExprP> pl = param_list();
        ws();
        if (lit(")")) {
          ExprP e(new Expr{Expr::OBJECT});
          e->id = name;
          e->params = std::move(pl);
          return e;
        }
      }
    }
    pos = save;
    if (ExprP e = string_lit()) return e;
    pos = save;
    std::string name;
    if (id(&name)) { ExprP e(new Expr{Expr::REF}); e->id = name; return e; }   // id_reference
    pos = save;
    return nullptr;
  }
  ExprP neg() {                       // neg_expression = { minus? ~ value }
    size_t save = pos;
    bool minus = false;
    if (at() == '-') { ++pos; minus = true; ws(); }
    ExprP v = value();
    if (!v) { pos = save; return nullptr; }
    if (!minus) return v;
    ExprP e(new Expr{Expr::MINUS});
    e->x = std::move(v);
    return e;
  }
  // Binary chains keep only the first operator/right operand (ast_node.rs:598-629).
  template <typename Sub>
  ExprP chain(Sub sub, const char* ops) {
    ExprP left = (this->*sub)();
    if (!left) return nullptr;
    ExprP result;
    for (;;) {
      size_t save = pos;
      ws();
      char c = at();
      if (!c || !strchr(ops, c)) { pos = save; break; }
      ++pos;
      ws();
      ExprP right = (this->*sub)();
      if (!right) { pos = save; break; }
      if (!result) {
        result.reset(new Expr{Expr::BINOP});
        result->op = c;
        result->x = std::move(left);
        result->y = std::move(right);
      }
    }
    return result ? std::move(result) : std::move(left);
  }
  ExprP mult() { return chain(&Parser::neg, "*/%"); }
  ExprP expression() { return chain(&Parser::mult, "+-"); }
  ExprP bool_expression() {           // { expression ~ bool_operator ~ expression }
    size_t save = pos;
    ExprP a = expression();
    if (!a) return nullptr;
    ws();
    char c = at();
    if (c != '<' && c != '>') { mark(); pos = save; return nullptr; }
    ++pos;
    ws();
    ExprP b = expression();
    if (!b) { pos = save; return nullptr; }
    ExprP e(new Expr{Expr::BINOP});
    e->op = c; e->x = std::move(a); e->y = std::move(b);
    return e;
  }

  StmtP statement() {                 // pest:17, alternatives in order
    size_t save = pos;
    if (lit("set") && ws1() && kw("camera")) {
      ws();
      if (lit("(")) {
        ws();
        ExprP e = expression();
        if (e) { ws(); if (lit(")")) { StmtP s(new Stmt{Stmt::CAMERA}); s->expr = std::move(e); return s; } }
      }
    }
    pos = save;
    if (lit("append") && ws1() && kw("light")) {
      ws();
      if (lit("(")) {
        ws();
        std::vector<ExprP> pl = param_list();
        ws();
        if (lit(")")) { StmtP s(new Stmt{Stmt::LIGHT}); s->params = std::move(pl); return s; }
      }
    }
    pos = save;
    if (kw("do")) {                   // do_statement lowers to its statement_list (ast_node.rs:383-394)
      ws();
      StmtP l = statement_list();
      ws();
      if (kw("end")) return l;
    }
    pos = save;
    for (int w = 0; w < 2; ++w) {     // if / while
      if (kw(w ? "while" : "if")) {
        ws();
        ExprP c = bool_expression();
        if (c) {
          ws();
          if (kw(w ? "do" : "then")) {
            ws();
            StmtP l = statement_list();
            ws();
            if (kw("end")) {
              StmtP s(new Stmt{w ? Stmt::WHILE : Stmt::IF});
              s->expr = std::move(c);
              s->body = l;
              return s;
            }
          }
        }
      }
      pos = save;
    }
    if (kw("call")) {
      ws();
      std::string name;
      if (id(&name)) {
        ws();
        if (lit("(")) {
          ws();
          std::vector<ExprP> pl = param_list();
          ws();
          if (lit(")")) { StmtP s(new Stmt{Stmt::CALL}); s->id = name; s->params = std::move(pl); return s; }
        }
      }
    }
    pos = save;
    if (kw("function")) {
      ws();
      std::string name;
      if (id(&name)) {
        ws();
        if (lit("(")) {
          std::vector<std::string> names;
          for (;;) {
            size_t s2 = pos;
            ws();
            std::string pn;
            if (!id(&pn)) { pos = s2; break; }
            names.push_back(pn);
            size_t s3 = pos; ws(); if (!lit(",")) pos = s3;
          }
          ws();
          if (lit(")")) {
            ws();
            StmtP l = statement_list();
            ws();
            if (kw("end")) {
              StmtP s(new Stmt{Stmt::FUNCTION});
              s->id = name; s->names = names; s->body = l;
              return s;
            }
          }
        }
      }
    }
    pos = save;
    if (const char* cmd = kw_any({"draw", "display", "append"})) {
      ws();
      if (lit("(")) {
        ws();
        std::vector<ExprP> pl = param_list();
        ws();
        if (lit(")")) {
          StmtP s(new Stmt{Stmt::DRAW});
          s->id = cmd;
          s->params = std::move(pl);
          if (s->id != "draw" && unimplemented.empty()) unimplemented = s->id;
          return s;
        }
      }
    }
    pos = save;
    {                                 // assignment_statement = { local_? ~ id ~ "=" ~ expression }
      bool local = false;
      if (kw("local")) { local = true; ws(); }
      std::string name;
      if (id(&name)) {
        ws();
        if (lit("=")) {
          ws();
          ExprP e = expression();
          if (e) {
            StmtP s(new Stmt{Stmt::ASSIGN});
            s->local = local; s->id = name; s->expr = std::move(e);
            return s;
          }
        }
      }
    }
    pos = save;
    if (const char* xf = kw_any({"scale", "rotate", "translate"})) {   // transformation_statement
      ws();
      if (lit("(")) {
        ExprP p[3];
        bool ok = true;
        for (int i = 0; i < 3 && ok; ++i) {
          ws();
          p[i] = expression();
          if (!p[i]) { ok = false; break; }
          ws();
          if (!lit(i < 2 ? "," : ")")) ok = false;
        }
        if (ok) {
          ws();
          StmtP body = statement();
          if (body) {
            StmtP s(new Stmt{Stmt::XFORM});
            s->x = std::move(p[0]); s->y = std::move(p[1]); s->z = std::move(p[2]);
            s->body = body;
            s->xform = xf[0];
            return s;
          }
        }
      }
    }
    pos = save;
    return nullptr;
  }
  StmtP statement_list() {            // statement_list = { statement* }
    StmtP l(new Stmt{Stmt::LIST});
    for (;;) {
      size_t save = pos;
      if (!l->list.empty()) ws();
      StmtP s = statement();
      if (!s) { pos = save; break; }
      l->list.push_back(s);
    }
    return l;
  }

 private:
  const char* s_;
  size_t n_;
};

// ------------------------------------------------------------------ evaluator
struct EvalError { int status; std::string msg; };

class Evaluator {
 public:
  Evaluator(rt_scene* scene, const char* asset_dir) : sc_(scene), asset_dir_(asset_dir ? asset_dir : "") {
    rt_transformation id;
    xf_identity(&id);
    xstack_.push_back(id);             // TransformationStack::new_with_identity
  }
  std::map<std::string, Value> globals;

  void exec(const Stmt& s) {
    switch (s.kind) {
      case Stmt::LIST:
        for (const StmtP& c : s.list) exec(*c);
        break;
      case Stmt::ASSIGN: {                                     // ast_node.rs:158-165
        Value v = eval(*s.expr);
        (s.local ? locals() : globals)[s.id] = v;
        break;
      }
      case Stmt::FUNCTION:                                     // :166-168
        functions_[s.id] = &s;
        break;
      case Stmt::CALL: {                                       // :169-175; context.rs:49-62
        std::vector<Value> vals;
        for (const ExprP& p : s.params) vals.push_back(eval(*p));
        auto it = functions_.find(s.id);
        if (it == functions_.end()) throw EvalError{RT_ERR_EVAL, "unknown function " + s.id};
        const Stmt& f = *it->second;
        if (f.names.size() != vals.size()) throw EvalError{RT_ERR_EVAL, "wrong argument count for " + s.id};
        frames_.emplace_back();
        for (size_t i = 0; i < vals.size(); ++i) frames_.back()[f.names[i]] = vals[i];
        exec(*f.body);
        frames_.pop_back();
        break;
      }
      case Stmt::DRAW: {                                       // :176-191
        std::vector<Value> vals;
        for (const ExprP& p : s.params) vals.push_back(eval(*p));
        if (vals.size() != 1) throw EvalError{RT_ERR_EVAL, "draw takes exactly one value"};
        if (vals[0].kind != Value::OBJECT) throw EvalError{RT_ERR_EVAL, "Didn't get an object on draw!"};
        draw(*vals[0].shape);
        break;
      }
      case Stmt::XFORM: {                                      // :192-219
        double x = number(eval(*s.x)), y = number(eval(*s.y)), z = number(eval(*s.z));
        rt_transformation t, composed;
        if (s.xform == 't') xf_translation(x, y, z, &t);
        else if (s.xform == 'r') xf_rotation(x, y, z, &t);
        else xf_scaling(x, y, z, &t);
        xf_compose(t, xstack_.back(), &composed);              // push_transformation (transformation.rs:21-28)
        xstack_.push_back(composed);
        exec(*s.body);
        xstack_.pop_back();
        break;
      }
      case Stmt::IF:
      case Stmt::WHILE:                                        // :220-229
        while (boolean(eval(*s.expr))) {
          exec(*s.body);
          if (s.kind == Stmt::IF) break;
        }
        break;
      case Stmt::LIGHT: {                                      // :230-251
        Bucket b = bucket(s.params);
        double col[4] = {0.5, 0.5, 0.5, 1.0};
        if (!b.colors.empty()) memcpy(col, b.colors[0].data(), sizeof col);
        double p[3] = {0, 0, 0};
        if (!b.vectors.empty()) memcpy(p, b.vectors[0].data(), sizeof p);
        double fade = b.numbers.empty() ? 100.0 : b.numbers[0];
        double wp[3];
        xf_apply(xstack_.back().matrix, p, wp);
        int rc = rt_scene_add_light(sc_, wp, col, fade);
        if (rc) throw EvalError{rc, rt_last_error()};
        break;
      }
      case Stmt::CAMERA: {                                     // :252-263 then raytracer.rs:289-299
        Value v = eval(*s.expr);
        if (v.kind != Value::VECTOR) throw EvalError{RT_ERR_EVAL, "Cannot convert value to vector"};
        double once[3], twice[3];
        xf_apply(xstack_.back().matrix, v.v, once);
        xf_apply(xstack_.back().matrix, once, twice);       // transformed a second time (quirk)
        rt_scene_set_camera(sc_, twice);
        break;
      }
    }
  }

 private:
  rt_scene* sc_;
  std::string asset_dir_;
  std::vector<rt_transformation> xstack_;
  std::vector<std::map<std::string, Value>> frames_;
  std::map<std::string, const Stmt*> functions_;
  std::map<std::string, int32_t> texture_cache_;

  std::map<std::string, Value>& locals() { return frames_.empty() ? globals : frames_.back(); }

  static double number(const Value& v) {
    if (v.kind != Value::NUMBER) throw EvalError{RT_ERR_EVAL, "Cannot convert value to number"};
    return v.num;
  }
  static bool boolean(const Value& v) {
    if (v.kind != Value::BOOLEAN) throw EvalError{RT_ERR_EVAL, "Cannot convert value to boolean"};
    return v.boolean;
  }

  struct Bucket {                                              // ValuesByType (ast_node.rs:105-148)
    std::vector<double> numbers;
    std::vector<std::string> strings;
    std::vector<std::array<double, 3>> vectors;
    std::vector<std::shared_ptr<const DslShape>> objects;
    std::vector<std::array<double, 4>> colors;
    std::vector<int32_t> textures;
  };
  Bucket bucket(const std::vector<ExprP>& params) {
    Bucket b;
    for (const ExprP& p : params) {
      Value v = eval(*p);
      switch (v.kind) {
        case Value::NUMBER: b.numbers.push_back(v.num); break;
        case Value::STRING: b.strings.push_back(v.str); break;
        case Value::COLOR: b.colors.push_back({v.c[0], v.c[1], v.c[2], v.c[3]}); break;
        case Value::VECTOR: b.vectors.push_back({v.v[0], v.v[1], v.v[2]}); break;
        case Value::OBJECT: b.objects.push_back(v.shape); break;
        case Value::TEXTURE: b.textures.push_back(v.texture); break;
        default: throw EvalError{RT_ERR_EVAL, "Unexpected argument type: boolean"};
      }
    }
    return b;
  }

  Value eval(const Expr& e) {
    switch (e.kind) {
      case Expr::VALUE: return e.value;
      case Expr::REF: {                                        // :442-451
        auto& l = locals();
        auto it = l.find(e.id);
        if (it != l.end()) return it->second;
        auto g = globals.find(e.id);
        if (g != globals.end()) return g->second;
        throw EvalError{RT_ERR_EVAL, "Didn't find variable " + e.id};
      }
      case Expr::VECTOR: {
        Value r;
        r.kind = Value::VECTOR;
        r.v[0] = number(eval(*e.x)); r.v[1] = number(eval(*e.y)); r.v[2] = number(eval(*e.z));
        return r;
      }
      case Expr::RGB: {
        Value r;
        r.kind = Value::COLOR;
        r.c[0] = number(eval(*e.x)); r.c[1] = number(eval(*e.y)); r.c[2] = number(eval(*e.z)); r.c[3] = 1.0;
        return r;
      }
      case Expr::OBJECT: return object(e);
      case Expr::TEXTURE: {                                    // :529-532
        Value f = eval(*e.x);
        if (f.kind != Value::STRING) throw EvalError{RT_ERR_EVAL, "Cannot convert value to string"};
        Value r;
        r.kind = Value::TEXTURE;
        r.texture = load_texture(f.str);
        return r;
      }
      case Expr::MINUS: {                                      // :533-542
        Value v = eval(*e.x);
        if (v.kind == Value::NUMBER) { v.num = -v.num; return v; }
        if (v.kind == Value::VECTOR) { for (double& c : v.v) c = -c; return v; }
        throw EvalError{RT_ERR_EVAL, "Cannot apply - to value"};
      }
      case Expr::BINOP: {                                      // :543-594
        Value a = eval(*e.x), b = eval(*e.y);
        Value r;
        switch (e.op) {
          case '+': r.kind = Value::NUMBER; r.num = number(a) + number(b); return r;
          case '-': r.kind = Value::NUMBER; r.num = number(a) - number(b); return r;
          case '*':
          case '/': {
            bool div = e.op == '/';
            if (a.kind == Value::NUMBER && b.kind == Value::NUMBER) {
              r.kind = Value::NUMBER; r.num = div ? a.num / b.num : a.num * b.num; return r;
            }
            const Value* num = a.kind == Value::NUMBER ? &a : b.kind == Value::NUMBER ? &b : nullptr;
            const Value* other = num == &a ? &b : &a;
            if (num && other->kind == Value::COLOR) {         // (Color, x) | (x, Color) -> colour op x
              r = *other;
              for (double& c : r.c) c = div ? c / num->num : c * num->num;
              return r;
            }
            if (num && other->kind == Value::VECTOR) {        // (Vector, x) | (x, Vector) -> vector op x
              r = *other;
              for (double& c : r.v) c = div ? c / num->num : c * num->num;
              return r;
            }
            throw EvalError{RT_ERR_EVAL, div ? "Cannot divide values" : "Cannot multiply values"};
          }
          case '<':
          case '>':
            if (a.kind != Value::NUMBER || b.kind != Value::NUMBER) throw EvalError{RT_ERR_EVAL, "Cannot compare values"};
            r.kind = Value::BOOLEAN;
            r.boolean = e.op == '<' ? a.num < b.num : a.num > b.num;
            return r;
          default:
            throw EvalError{RT_ERR_EVAL, "Operator Modulo not yet implemented"};
        }
      }
    }
    throw EvalError{RT_ERR_EVAL, "bad expression"};
  }

  Value object(const Expr& e) {                                // :466-528
    Bucket b = bucket(e.params);
    size_t in = 0, is = 0, iv = 0, io = 0, ic = 0, it = 0;
    auto s = std::make_shared<DslShape>();
    if (e.id == "sphere" || e.id == "cube") {
      s->kind = e.id == "sphere" ? DslShape::SPHERE : DslShape::CUBE;
      if (iv < b.vectors.size()) { memcpy(s->center, b.vectors[iv].data(), sizeof s->center); ++iv; }
      s->size = in < b.numbers.size() ? b.numbers[in++] : 1.0;
    } else if (e.id == "plane") {
      s->kind = DslShape::PLANE;
      if (iv < b.vectors.size()) { memcpy(s->normal, b.vectors[iv].data(), sizeof s->normal); ++iv; }
      s->distance = in < b.numbers.size() ? b.numbers[in++] : 1.0;
    } else {
      s->kind = DslShape::CSG;
      std::string op = is < b.strings.size() ? b.strings[is++] : "union";
      if (op == "union") s->op = RT_CSG_UNION;
      else if (op == "intersection") s->op = RT_CSG_INTERSECTION;
      else if (op == "difference") s->op = RT_CSG_DIFFERENCE;
      else throw EvalError{RT_ERR_EVAL, "Unknown CSG operator: " + op};
      if (io >= b.objects.size()) throw EvalError{RT_ERR_EVAL, "Expected object 1!"};
      s->a = b.objects[io++];
      if (io >= b.objects.size()) throw EvalError{RT_ERR_EVAL, "Expected object 2!"};
      s->b = b.objects[io++];
    }
    s->t = xstack_.back();
    if (it < b.textures.size()) { s->textured = true; s->texture = b.textures[it++]; }
    else if (ic < b.colors.size()) { memcpy(s->color, b.colors[ic].data(), sizeof s->color); ++ic; }
    s->reflectivity = in < b.numbers.size() ? b.numbers[in++] : 0.0;
    s->transparency = in < b.numbers.size() ? b.numbers[in++] : 0.0;
    if (in != b.numbers.size() || is != b.strings.size() || iv != b.vectors.size() ||
        io != b.objects.size() || ic != b.colors.size() || it != b.textures.size())
      throw EvalError{RT_ERR_EVAL, "assertion failed: unused arguments to " + e.id};   // assert_empty
    Value r;
    r.kind = Value::OBJECT;
    r.shape = s;
    return r;
  }

  // Shape::to_rt_object (sceneparser/shape.rs:42-93)
  int32_t lower(const DslShape& s) {
    int rc;
    switch (s.kind) {
      case DslShape::SPHERE: rc = rt_shape_sphere(sc_, &s.t, s.center, s.size); break;
      case DslShape::CUBE: rc = rt_shape_cube(sc_, &s.t, s.center, s.size); break;
      case DslShape::PLANE: rc = rt_shape_plane(sc_, &s.t, s.normal, s.distance); break;
      default: {
        int32_t a = lower(*s.a);
        int32_t b = lower(*s.b);
        rc = rt_shape_csg(sc_, s.op, a, b);
      }
    }
    if (rc < 0) throw EvalError{rc, rt_last_error()};
    return rc;
  }
  void draw(const DslShape& s) {
    int32_t id = lower(s);
    rt_material m;
    memset(&m, 0, sizeof m);
    memcpy(m.color, s.color, sizeof m.color);
    m.texture = s.textured ? s.texture : -1;
    m.reflectivity = s.reflectivity;
    m.transparency = s.transparency;
    int rc = rt_scene_add_object(sc_, id, &m);
    if (rc) throw EvalError{rc, rt_last_error()};
  }

  // Texture::from_file (sceneparser/texture.rs:20-40), path relative to asset_dir.  The file is read
  // every time (as the reference reads it); its decoded pixels come from decoded_png, keyed by the file's
  // bytes, so a host that rebuilds the scene every frame (debug_window.rs:53-68) decodes it once.
  int32_t load_texture(const std::string& name) {
    auto c = texture_cache_.find(name);
    if (c != texture_cache_.end()) return c->second;
    std::string path = (asset_dir_.empty() || name.empty() || name[0] == '/') ? name : asset_dir_ + "/" + name;
    std::vector<uint8_t> file;
    if (!read_file(path, &file)) throw EvalError{RT_ERR_IO, "cannot read texture " + path};
    std::shared_ptr<const DecodedPng> img = decoded_png(file);
    if (!img) throw EvalError{RT_ERR_IO, std::string("cannot decode texture ") + path + ": " + rt_last_error()};
    int id = rt_scene_add_texture(sc_, img->w, img->h, img->rgba.data());
    if (id < 0) throw EvalError{id, rt_last_error()};
    texture_cache_[name] = id;
    return id;
  }
};

}  // namespace

int compile_scene_text(const char* text, const char* asset_dir, double time, rt_scene* scene) {
  Parser p(text);
  p.ws();                                                      // scene = _{ SOI ~ statement_list ~ EOI }
  StmtP ast = p.statement_list();
  p.ws();
  if (!p.eof()) {
    size_t at = p.furthest > p.pos ? p.furthest : p.pos;
    int line = 1;
    for (size_t i = 0; i < at && text[i]; ++i) line += text[i] == '\n';
    return fail(RT_ERR_PARSE, "scene parse error near line %d (offset %zu)", line, at);
  }
  if (!p.unimplemented.empty())                                // from_pest panics before executing
    return fail(RT_ERR_EVAL, "not implemented: command '%s'", p.unimplemented.c_str());
  try {
    Evaluator ev(scene, asset_dir);
    Value t;
    t.kind = Value::NUMBER;
    t.num = time;
    ev.globals["time"] = t;                                    // scene_loader.rs:34
    ev.exec(*ast);
  } catch (const EvalError& e) {
    return fail(e.status, "%s", e.msg.c_str());
  } catch (const std::exception& e) {
    return fail(RT_ERR_NOMEM, "%s", e.what());
  }
  return RT_OK;
}

}  // namespace rt
