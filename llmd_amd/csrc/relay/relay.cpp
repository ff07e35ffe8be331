// llmd-relay: the router's native data plane (SURVEY C07 proxy / N17 Envoy).
//
// The reference puts Envoy (C++) in the data path and the EPP beside it: Envoy
// holds the client and upstream connections and relays the response stream, the
// EPP only decides (guides/no-kubernetes-deployment/README.md:205-218 runs the
// standalone proxy with --concurrency 8 worker threads). This is that split for
// one node: N epoll threads (one listening socket each, SO_REUSEPORT, so the
// kernel spreads client connections over them) relay HTTP/1.1 requests and their
// streamed responses, and ask the ONE EPP process (llmd_amd/router/workers.py
// EppServer, single writer of all scheduling state) for each decision over a Unix
// socket with the workers' protocol: 4-byte big-endian length + msgpack map
//   -> {"op":"pick","id","path","headers","body"}   <- {"id","d":{tok,endpoint,headers,body,request_id,stream}}
//                                                       or {"id","err":{status,msg,reason}}
//   -> {"op":"hdr","tok","status","headers"}  -> {"op":"chunk","tok","chunk","t"} (only when asked)
//   -> {"op":"done","tok","info":{status,ttft,tpot,duration,usage}}
//   -> {"op":"state","id"}                     <- {"id","eps","health":[status,text],"chunks"}
// so response hooks (prefix-cache confirmation, predictor training, SLO metrics,
// flow control) run in the EPP exactly as behind the Python proxy (router/proxy.py).
//
// Per request a thread does no allocation-heavy work beyond the header vectors:
// upstream response bytes are forwarded verbatim (chunked framing included), the
// chunk parser only tracks framing and keeps a 64 KB payload tail from which the
// usage block is parsed once, at the end. Upstream connections are kept alive in
// a per-thread pool per endpoint.
//
// Semantics follow router/proxy.py: FailOpen / FailClose on EPP failure, EPP
// rejections keep their status and x-llm-d-request-dropped-reason, 502 on an
// upstream failure before the response head, HA standby answers 503.
//
//   llmd-relay --port P --uds PATH [--host H] [--threads N] [--failure-mode FailOpen|FailClose]
#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <random>
#include <string>
#include <thread>
#include <unordered_map>
#include <utility>
#include <vector>

namespace {

double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);  // the clock of Python's time.monotonic(), shared with the EPP
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

std::string lower(std::string s) {
  for (auto& c : s) c = (char)tolower((unsigned char)c);
  return s;
}

bool ieq(const std::string& a, const char* b) {
  size_t n = strlen(b);
  if (a.size() != n) return false;
  for (size_t i = 0; i < n; ++i)
    if (tolower((unsigned char)a[i]) != tolower((unsigned char)b[i])) return false;
  return true;
}

// ------------------------------------------------------------------ values (msgpack / JSON)
struct Val {
  enum T { NIL, BOOL, INT, DBL, STR, BIN, ARR, MAP } t = NIL;
  bool b = false;
  int64_t i = 0;
  double d = 0;
  std::string s;  // STR and BIN
  std::vector<Val> a;
  std::vector<std::pair<std::string, Val>> m;
  const Val* get(const char* k) const {
    if (t != MAP) return nullptr;
    for (auto& kv : m)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  int64_t as_int(int64_t dflt = 0) const { return t == INT ? i : t == DBL ? (int64_t)d : dflt; }
  double as_dbl() const { return t == DBL ? d : t == INT ? (double)i : 0.0; }
  bool truthy() const {
    switch (t) {
      case NIL: return false;
      case BOOL: return b;
      case INT: return i != 0;
      case DBL: return d != 0;
      case STR: case BIN: return !s.empty();
      case ARR: return !a.empty();
      case MAP: return !m.empty();
    }
    return false;
  }
};

// msgpack writer
struct Pk {
  std::string& o;
  explicit Pk(std::string& out) : o(out) {}
  void u8(uint8_t v) { o.push_back((char)v); }
  void be(uint64_t v, int n) {
    for (int k = n - 1; k >= 0; --k) o.push_back((char)((v >> (8 * k)) & 0xff));
  }
  void nil() { u8(0xc0); }
  void boolean(bool v) { u8(v ? 0xc3 : 0xc2); }
  void integer(int64_t v) {
    if (v >= 0 && v < 128) u8((uint8_t)v);
    else if (v < 0 && v >= -32) u8((uint8_t)(0xe0 | (v + 32)));
    else { u8(0xd3); be((uint64_t)v, 8); }
  }
  void dbl(double v) {
    uint64_t bits;
    memcpy(&bits, &v, 8);
    u8(0xcb);
    be(bits, 8);
  }
  void str(const char* p, size_t n) {
    if (n < 32) u8((uint8_t)(0xa0 | n));
    else if (n < 256) { u8(0xd9); be(n, 1); }
    else if (n < 65536) { u8(0xda); be(n, 2); }
    else { u8(0xdb); be(n, 4); }
    o.append(p, n);
  }
  void str(const std::string& s) { str(s.data(), s.size()); }
  void str(const char* s) { str(s, strlen(s)); }
  void bin(const char* p, size_t n) {
    if (n < 256) { u8(0xc4); be(n, 1); }
    else if (n < 65536) { u8(0xc5); be(n, 2); }
    else { u8(0xc6); be(n, 4); }
    o.append(p, n);
  }
  void map(size_t n) {
    if (n < 16) u8((uint8_t)(0x80 | n));
    else if (n < 65536) { u8(0xde); be(n, 2); }
    else { u8(0xdf); be(n, 4); }
  }
  void arr(size_t n) {
    if (n < 16) u8((uint8_t)(0x90 | n));
    else if (n < 65536) { u8(0xdc); be(n, 2); }
    else { u8(0xdd); be(n, 4); }
  }
  void val(const Val& v) {
    switch (v.t) {
      case Val::NIL: nil(); break;
      case Val::BOOL: boolean(v.b); break;
      case Val::INT: integer(v.i); break;
      case Val::DBL: dbl(v.d); break;
      case Val::STR: str(v.s); break;
      case Val::BIN: bin(v.s.data(), v.s.size()); break;
      case Val::ARR:
        arr(v.a.size());
        for (auto& x : v.a) val(x);
        break;
      case Val::MAP:
        map(v.m.size());
        for (auto& kv : v.m) {
          str(kv.first);
          val(kv.second);
        }
        break;
    }
  }
};

// msgpack reader (the subset the EPP sends; map keys read as strings)
struct Up {
  const uint8_t* p;
  const uint8_t* e;
  bool ok = true;
  uint64_t be(int n) {
    if (e - p < n) { ok = false; return 0; }
    uint64_t v = 0;
    for (int k = 0; k < n; ++k) v = (v << 8) | p[k];
    p += n;
    return v;
  }
  void bytes(std::string& out, size_t n) {
    if ((size_t)(e - p) < n) { ok = false; return; }
    out.assign((const char*)p, n);
    p += n;
  }
  void read(Val& v, int depth = 0) {
    if (!ok || p >= e || depth > 32) { ok = false; return; }
    uint8_t c = *p++;
    if (c <= 0x7f) { v.t = Val::INT; v.i = c; return; }
    if (c >= 0xe0) { v.t = Val::INT; v.i = (int8_t)c; return; }
    if ((c & 0xf0) == 0x80) return read_map(v, c & 0x0f, depth);
    if ((c & 0xf0) == 0x90) return read_arr(v, c & 0x0f, depth);
    if ((c & 0xe0) == 0xa0) { v.t = Val::STR; bytes(v.s, c & 0x1f); return; }
    switch (c) {
      case 0xc0: v.t = Val::NIL; return;
      case 0xc2: v.t = Val::BOOL; v.b = false; return;
      case 0xc3: v.t = Val::BOOL; v.b = true; return;
      case 0xc4: v.t = Val::BIN; bytes(v.s, be(1)); return;
      case 0xc5: v.t = Val::BIN; bytes(v.s, be(2)); return;
      case 0xc6: v.t = Val::BIN; bytes(v.s, be(4)); return;
      case 0xca: {
        uint32_t b = (uint32_t)be(4);
        float f;
        memcpy(&f, &b, 4);
        v.t = Val::DBL; v.d = f;
        return;
      }
      case 0xcb: {
        uint64_t b = be(8);
        v.t = Val::DBL;
        memcpy(&v.d, &b, 8);
        return;
      }
      case 0xcc: v.t = Val::INT; v.i = (int64_t)be(1); return;
      case 0xcd: v.t = Val::INT; v.i = (int64_t)be(2); return;
      case 0xce: v.t = Val::INT; v.i = (int64_t)be(4); return;
      case 0xcf: v.t = Val::INT; v.i = (int64_t)be(8); return;
      case 0xd0: v.t = Val::INT; v.i = (int8_t)be(1); return;
      case 0xd1: v.t = Val::INT; v.i = (int16_t)be(2); return;
      case 0xd2: v.t = Val::INT; v.i = (int32_t)be(4); return;
      case 0xd3: v.t = Val::INT; v.i = (int64_t)be(8); return;
      case 0xd9: v.t = Val::STR; bytes(v.s, be(1)); return;
      case 0xda: v.t = Val::STR; bytes(v.s, be(2)); return;
      case 0xdb: v.t = Val::STR; bytes(v.s, be(4)); return;
      case 0xdc: return read_arr(v, be(2), depth);
      case 0xdd: return read_arr(v, be(4), depth);
      case 0xde: return read_map(v, be(2), depth);
      case 0xdf: return read_map(v, be(4), depth);
      default: ok = false;
    }
  }
  void read_arr(Val& v, size_t n, int depth) {
    v.t = Val::ARR;
    if (n > (size_t)(e - p)) { ok = false; return; }
    v.a.resize(n);
    for (auto& x : v.a) read(x, depth + 1);
  }
  void read_map(Val& v, size_t n, int depth) {
    v.t = Val::MAP;
    if (n > (size_t)(e - p)) { ok = false; return; }
    v.m.resize(n);
    for (auto& kv : v.m) {
      Val k;
      read(k, depth + 1);
      if (k.t == Val::STR || k.t == Val::BIN) kv.first = std::move(k.s);
      else if (k.t == Val::INT) kv.first = std::to_string(k.i);
      read(kv.second, depth + 1);
    }
  }
};

// JSON -> Val (for the usage block of the response tail)
struct Js {
  const char* p;
  const char* e;
  bool ok = true;
  void ws() {
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  }
  static void utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) o.push_back((char)cp);
    else if (cp < 0x800) { o.push_back((char)(0xc0 | (cp >> 6))); o.push_back((char)(0x80 | (cp & 0x3f))); }
    else if (cp < 0x10000) {
      o.push_back((char)(0xe0 | (cp >> 12)));
      o.push_back((char)(0x80 | ((cp >> 6) & 0x3f)));
      o.push_back((char)(0x80 | (cp & 0x3f)));
    } else {
      o.push_back((char)(0xf0 | (cp >> 18)));
      o.push_back((char)(0x80 | ((cp >> 12) & 0x3f)));
      o.push_back((char)(0x80 | ((cp >> 6) & 0x3f)));
      o.push_back((char)(0x80 | (cp & 0x3f)));
    }
  }
  uint32_t hex4() {
    if (e - p < 4) { ok = false; return 0; }
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {
      char c = p[k];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else { ok = false; return 0; }
    }
    p += 4;
    return v;
  }
  void string(std::string& o) {
    ++p;  // opening quote
    while (p < e && *p != '"') {
      if (*p == '\\') {
        if (++p >= e) { ok = false; return; }
        char c = *p++;
        switch (c) {
          case 'n': o.push_back('\n'); break;
          case 't': o.push_back('\t'); break;
          case 'r': o.push_back('\r'); break;
          case 'b': o.push_back('\b'); break;
          case 'f': o.push_back('\f'); break;
          case 'u': {
            uint32_t cp = hex4();
            if (cp >= 0xd800 && cp < 0xdc00 && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
              p += 2;
              uint32_t lo = hex4();
              cp = 0x10000 + ((cp - 0xd800) << 10) + (lo - 0xdc00);
            }
            utf8(o, cp);
            break;
          }
          default: o.push_back(c);
        }
      } else {
        o.push_back(*p++);
      }
    }
    if (p >= e) { ok = false; return; }
    ++p;
  }
  void value(Val& v, int depth = 0) {
    ws();
    if (p >= e || depth > 32) { ok = false; return; }
    char c = *p;
    if (c == '{') {
      ++p;
      v.t = Val::MAP;
      ws();
      if (p < e && *p == '}') { ++p; return; }
      while (ok) {
        ws();
        if (p >= e || *p != '"') { ok = false; return; }
        std::pair<std::string, Val> kv;
        string(kv.first);
        ws();
        if (p >= e || *p != ':') { ok = false; return; }
        ++p;
        value(kv.second, depth + 1);
        v.m.push_back(std::move(kv));
        ws();
        if (p < e && *p == ',') { ++p; continue; }
        if (p < e && *p == '}') { ++p; return; }
        ok = false;
      }
    } else if (c == '[') {
      ++p;
      v.t = Val::ARR;
      ws();
      if (p < e && *p == ']') { ++p; return; }
      while (ok) {
        v.a.emplace_back();
        value(v.a.back(), depth + 1);
        ws();
        if (p < e && *p == ',') { ++p; continue; }
        if (p < e && *p == ']') { ++p; return; }
        ok = false;
      }
    } else if (c == '"') {
      v.t = Val::STR;
      string(v.s);
    } else if (e - p >= 4 && !strncmp(p, "true", 4)) { v.t = Val::BOOL; v.b = true; p += 4; }
    else if (e - p >= 5 && !strncmp(p, "false", 5)) { v.t = Val::BOOL; v.b = false; p += 5; }
    else if (e - p >= 4 && !strncmp(p, "null", 4)) { v.t = Val::NIL; p += 4; }
    else {
      const char* s = p;
      bool flt = false;
      while (p < e && (isdigit((unsigned char)*p) || *p == '-' || *p == '+' || *p == '.' || *p == 'e' || *p == 'E')) {
        if (*p == '.' || *p == 'e' || *p == 'E') flt = true;
        ++p;
      }
      if (p == s) { ok = false; return; }
      std::string num(s, p - s);
      if (flt) { v.t = Val::DBL; v.d = strtod(num.c_str(), nullptr); }
      else { v.t = Val::INT; v.i = strtoll(num.c_str(), nullptr, 10); }
    }
  }
};

bool parse_json(const char* p, size_t n, Val& out) {
  Js j{p, p + n};
  j.value(out);
  return j.ok;
}

// usage from the tail of a JSON or SSE response (router/proxy.py _find_usage)
bool find_usage(const std::string& tail, Val& usage) {
  size_t a = 0;
  while (a < tail.size() && isspace((unsigned char)tail[a])) ++a;
  if (a < tail.size() && tail[a] == '{') {
    Val v;
    if (parse_json(tail.data() + a, tail.size() - a, v)) {
      const Val* u = v.get("usage");
      if (u && u->t == Val::MAP) { usage = *u; return true; }
      return false;
    }
  }
  size_t end = tail.size();
  while (end > 0) {
    size_t nl = tail.rfind('\n', end - 1);
    size_t beg = nl == std::string::npos ? 0 : nl + 1;
    std::string line = tail.substr(beg, end - beg);
    end = nl == std::string::npos ? 0 : nl;
    size_t s = 0, t = line.size();
    while (s < t && isspace((unsigned char)line[s])) ++s;
    while (t > s && isspace((unsigned char)line[t - 1])) --t;
    if (t - s < 5 || line.compare(s, 5, "data:") != 0) continue;
    if (line.find("usage", s) == std::string::npos) continue;
    Val v;
    if (!parse_json(line.data() + s + 5, t - s - 5, v)) continue;
    const Val* u = v.get("usage");
    if (u && u->t == Val::MAP && u->truthy()) { usage = *u; return true; }
  }
  return false;
}

// ------------------------------------------------------------------ HTTP
using Headers = std::vector<std::pair<std::string, std::string>>;

const std::string* hget(const Headers& h, const char* name) {
  for (auto& kv : h)
    if (ieq(kv.first, name)) return &kv.second;
  return nullptr;
}

bool hop_header(const std::string& k) {
  return ieq(k, "host") || ieq(k, "content-length") || ieq(k, "transfer-encoding") || ieq(k, "connection") ||
         ieq(k, "keep-alive");
}

// RFC 9110 tchar: the only bytes a field name may hold
bool tchar(unsigned char ch) {
  if (ch >= '0' && ch <= '9') return true;
  if ((ch | 0x20) >= 'a' && (ch | 0x20) <= 'z') return true;
  return strchr("!#$%&'*+-.^_`|~", ch) != nullptr && ch != 0;
}

// parse "Name: value\r\n" lines of [p, e) (the head without its first line).
// Strict per RFC 9112: the name is a non-empty token with nothing
// between it and the colon ("Content-Length :" would slip past hop_header and
// reach the upstream as a second framing header), no obs-fold continuation
// lines, and no bare CR or NUL in a value. Any of those -> 400.
bool parse_headers(const char* p, const char* e, Headers& out) {
  while (p < e) {
    const char* nl = (const char*)memchr(p, '\n', e - p);
    const char* le = nl ? nl : e;
    const char* ln_end = (le > p && le[-1] == '\r') ? le - 1 : le;
    if (ln_end > p) {
      const char* colon = (const char*)memchr(p, ':', ln_end - p);
      if (!colon || colon == p) return false;
      for (const char* q = p; q < colon; ++q)
        if (!tchar((unsigned char)*q)) return false;
      for (const char* q = colon + 1; q < ln_end; ++q)
        if (*q == '\r' || *q == '\0') return false;
      const char* v = colon + 1;
      while (v < ln_end && (*v == ' ' || *v == '\t')) ++v;
      const char* ve = ln_end;
      while (ve > v && (ve[-1] == ' ' || ve[-1] == '\t')) --ve;
      out.emplace_back(std::string(p, colon - p), std::string(v, ve - v));
    }
    p = nl ? nl + 1 : e;
  }
  return true;
}

const char* reason(int st) {
  switch (st) {
    case 200: return "OK";
    case 201: return "Created";
    case 204: return "No Content";
    case 400: return "Bad Request";
    case 401: return "Unauthorized";
    case 403: return "Forbidden";
    case 404: return "Not Found";
    case 408: return "Request Timeout";
    case 413: return "Payload Too Large";
    case 429: return "Too Many Requests";
    case 500: return "Internal Server Error";
    case 502: return "Bad Gateway";
    case 503: return "Service Unavailable";
    case 504: return "Gateway Timeout";
    default: return "Status";
  }
}

// chunked transfer-coding framing tracker: payload bytes go to a callback
struct Chunked {
  enum St { SIZE, DATA, DATA_END, TRAILER, DONE } st = SIZE;
  uint64_t left = 0;
  std::string line;
  // consumes from [p, e); returns bytes consumed or -1 on a framing error
  template <class F>
  long feed(const char* p, const char* e, F&& on_data) {
    const char* s = p;
    while (p < e && st != DONE) {
      if (st == DATA) {
        size_t n = (size_t)std::min<uint64_t>(left, (uint64_t)(e - p));
        on_data(p, n);
        p += n;
        left -= n;
        if (left == 0) st = DATA_END;
        continue;
      }
      const char* nl = (const char*)memchr(p, '\n', e - p);
      if (!nl) {
        line.append(p, e - p);
        if (line.size() > 8192) return -1;
        p = e;
        break;
      }
      line.append(p, nl - p);
      p = nl + 1;
      if (!line.empty() && line.back() == '\r') line.pop_back();
      if (st == SIZE) {
        char* end = nullptr;
        unsigned long long n = strtoull(line.c_str(), &end, 16);
        if (end == line.c_str()) return -1;
        left = n;
        st = n == 0 ? TRAILER : DATA;
      } else if (st == DATA_END) {
        if (!line.empty()) return -1;
        st = SIZE;
      } else if (st == TRAILER) {
        if (line.empty()) st = DONE;
      }
      line.clear();
    }
    return p - s;
  }
};

const char* const INFERENCE_PATHS[] = {"/v1/completions", "/v1/chat/completions", "/v1/embeddings", "/v1/responses",
                                       "/v1/conversations", "/v1/messages", "/inference/v1/generate",
                                       "/vllm.grpc.engine.VllmEngine/Generate", "/vllm.grpc.engine.VllmEngine/Embed"};

bool inference_path(const std::string& p) {
  for (auto* q : INFERENCE_PATHS)
    if (p == q) return true;
  return false;
}

void set_nonblock(int fd) { fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK); }

// ------------------------------------------------------------------ loop objects
enum Kind { K_LISTEN, K_CLIENT, K_UP, K_EPP };

struct Ev {
  Kind kind;
  int fd = -1;
  uint32_t events = 0;
};

struct Client;
struct Upstream;

struct Exchange {
  // request
  std::string method, target, path;
  Headers hdrs;
  std::string body;
  bool keep_alive = true;
  bool inference = false;
  // decision
  int64_t tok = 0;  // 0: no EPP decision (passthrough / fail-open)
  std::string endpoint, request_id;
  bool stream = false;
  Headers extra;
  bool has_body_override = false;
  std::string body_override;
  // response
  Upstream* up = nullptr;
  bool retried = false;
  bool head_sent = false;  // client saw the response head
  int status = 0;
  enum Framing { F_LEN, F_CHUNKED, F_CLOSE, F_NONE } framing = F_NONE;
  uint64_t remaining = 0;
  Chunked chunked;
  bool rechunk = false;  // close-delimited upstream relayed with chunked framing
  bool up_keep = true;
  double t0 = 0, first = -1, last = -1;
  std::string tail;
  bool finished = false;
};

struct Client : Ev {
  uint64_t id = 0;
  std::string in, out;
  size_t out_off = 0;
  std::unique_ptr<Exchange> ex;
  bool close_after = false;
  bool dead = false;
  bool sent_continue = false;
  // chunked request body: parser state kept across reads, so each byte is
  // decoded once (not re-parsed from the start whenever more data arrives)
  Chunked req_ck;
  std::string req_body;
  size_t req_fed = 0;  // bytes after the head already given to req_ck
};

struct Upstream : Ev {
  std::string key;
  std::string in, out;
  size_t out_off = 0;
  Client* client = nullptr;  // owner while in use
  bool connecting = false;
  bool reused = false;
  bool got_bytes = false;
  double t_conn = 0;
};

struct Epp : Ev {
  std::string in, out;
  size_t out_off = 0;
};

struct Options {
  std::string host = "0.0.0.0", uds;
  int port = 0, threads = 4;
  bool fail_open = true;
};

constexpr size_t HIGH_WATER = 4u << 20, LOW_WATER = 1u << 20;

class Loop {
 public:
  explicit Loop(const Options& o, int idx) : opt_(o), rng_(std::random_device{}() ^ (idx * 0x9e3779b9u)) {}

  int run() {
    ep_ = epoll_create1(0);
    if (ep_ < 0) return perror("epoll_create1"), 1;
    if (!listen_()) return 1;
    connect_epp();
    std::vector<epoll_event> evs(256);
    double next_state = 0;
    while (true) {
      int n = epoll_wait(ep_, evs.data(), (int)evs.size(), 50);
      if (n < 0 && errno != EINTR) return perror("epoll_wait"), 1;
      for (int k = 0; k < n; ++k) dispatch((Ev*)evs[k].data.ptr, evs[k].events);
      reap();
      double t = now_s();
      if (t >= next_state) {
        next_state = t + 0.5;
        if (epp_ == nullptr) connect_epp();
        else send_state();
      }
      check_connect_timeouts(t);
    }
  }

 private:
  const Options& opt_;
  std::mt19937_64 rng_;
  int ep_ = -1;
  Ev lis_{K_LISTEN};
  Epp* epp_ = nullptr;
  uint64_t next_id_ = 1;
  uint64_t next_client_ = 1;
  std::unordered_map<uint64_t, Client*> clients_;
  std::unordered_map<uint64_t, uint64_t> pending_;  // pick id -> client id
  std::unordered_map<std::string, std::vector<Upstream*>> pool_;
  std::vector<Upstream*> connecting_;
  std::vector<Ev*> graveyard_;
  std::unordered_map<std::string, sockaddr_storage> addr_cache_;
  // EPP state
  std::vector<std::string> eps_;
  int health_status_ = 503;
  std::string health_text_ = "connecting";
  bool chunks_ = false;

  // ---------------------------------------------------------------- epoll plumbing
  void add(Ev* e, uint32_t ev) {
    epoll_event x{};
    x.events = ev;
    x.data.ptr = e;
    e->events = ev;
    epoll_ctl(ep_, EPOLL_CTL_ADD, e->fd, &x);
  }
  void mod(Ev* e, uint32_t ev) {
    if (e->events == ev || e->fd < 0) return;
    epoll_event x{};
    x.events = ev;
    x.data.ptr = e;
    e->events = ev;
    epoll_ctl(ep_, EPOLL_CTL_MOD, e->fd, &x);
  }
  void drop(Ev* e) {
    if (e->fd >= 0) {
      epoll_ctl(ep_, EPOLL_CTL_DEL, e->fd, nullptr);
      close(e->fd);
      e->fd = -1;
    }
    graveyard_.push_back(e);
  }
  void reap() {
    for (Ev* e : graveyard_) {
      switch (e->kind) {
        case K_CLIENT: delete static_cast<Client*>(e); break;
        case K_UP: delete static_cast<Upstream*>(e); break;
        case K_EPP: delete static_cast<Epp*>(e); break;
        default: break;
      }
    }
    graveyard_.clear();
  }

  bool listen_() {
    int fd = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK, 0);
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    setsockopt(fd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(opt_.port);
    if (inet_pton(AF_INET, opt_.host.c_str(), &a.sin_addr) != 1) a.sin_addr.s_addr = INADDR_ANY;
    if (bind(fd, (sockaddr*)&a, sizeof a) < 0 || listen(fd, 4096) < 0) {
      perror("llmd-relay: bind/listen");
      close(fd);
      return false;
    }
    lis_.fd = fd;
    add(&lis_, EPOLLIN);
    return true;
  }

  void dispatch(Ev* e, uint32_t ev) {
    if (e->fd < 0) return;  // dropped earlier in this batch
    switch (e->kind) {
      case K_LISTEN: accept_all(); break;
      case K_CLIENT: on_client(static_cast<Client*>(e), ev); break;
      case K_UP: on_upstream(static_cast<Upstream*>(e), ev); break;
      case K_EPP: on_epp(ev); break;
    }
  }

  // generic non-blocking write of out[off:]; false on a hard error
  static bool flush(int fd, std::string& out, size_t& off) {
    while (off < out.size()) {
      ssize_t n = send(fd, out.data() + off, out.size() - off, MSG_NOSIGNAL);
      if (n < 0) {
        if (errno == EAGAIN || errno == EWOULDBLOCK) break;
        if (errno == EINTR) continue;
        return false;
      }
      off += (size_t)n;
    }
    if (off == out.size()) {
      out.clear();
      off = 0;
    } else if (off > (1u << 20)) {
      out.erase(0, off);
      off = 0;
    }
    return true;
  }
  // read everything available into buf; returns 0 on EOF, -1 on error, 1 otherwise
  static int slurp(int fd, std::string& buf) {
    char tmp[65536];
    while (true) {
      ssize_t n = recv(fd, tmp, sizeof tmp, 0);
      if (n > 0) {
        buf.append(tmp, (size_t)n);
        if ((size_t)n < sizeof tmp) return 1;
        continue;
      }
      if (n == 0) return 0;
      if (errno == EAGAIN || errno == EWOULDBLOCK) return 1;
      if (errno == EINTR) continue;
      return -1;
    }
  }

  // ---------------------------------------------------------------- EPP connection
  void connect_epp() {
    int fd = socket(AF_UNIX, SOCK_STREAM, 0);
    sockaddr_un a{};
    a.sun_family = AF_UNIX;
    strncpy(a.sun_path, opt_.uds.c_str(), sizeof a.sun_path - 1);
    if (connect(fd, (sockaddr*)&a, sizeof a) < 0) {
      close(fd);
      if (health_text_ != "connecting") { health_status_ = 503; health_text_ = "EPP connection lost"; }
      return;
    }
    set_nonblock(fd);
    epp_ = new Epp();
    epp_->kind = K_EPP;
    epp_->fd = fd;
    add(epp_, EPOLLIN);
    send_state();
  }

  void epp_send(const std::string& payload) {
    if (epp_ == nullptr) return;
    uint32_t n = htonl((uint32_t)payload.size());
    epp_->out.append((const char*)&n, 4);
    epp_->out.append(payload);
    if (!flush(epp_->fd, epp_->out, epp_->out_off)) return epp_lost();
    mod(epp_, EPOLLIN | (epp_->out.empty() ? 0u : (uint32_t)EPOLLOUT));
  }

  void send_state() {
    std::string m;
    Pk pk(m);
    pk.map(2);
    pk.str("op"); pk.str("state");
    pk.str("id"); pk.integer((int64_t)next_id_++);
    epp_send(m);
  }

  void epp_lost() {
    if (epp_ == nullptr) return;
    drop(epp_);
    epp_ = nullptr;
    health_status_ = 503;
    health_text_ = "EPP connection lost";
    // every pick in flight fails over like an EPP error (FailOpen / FailClose)
    auto pend = std::move(pending_);
    pending_.clear();
    for (auto& kv : pend) {
      auto it = clients_.find(kv.second);
      if (it != clients_.end() && it->second->ex) epp_failed(it->second, "EPP connection lost");
    }
  }

  void on_epp(uint32_t ev) {
    if (ev & EPOLLOUT) {
      if (!flush(epp_->fd, epp_->out, epp_->out_off)) return epp_lost();
      mod(epp_, EPOLLIN | (epp_->out.empty() ? 0u : (uint32_t)EPOLLOUT));
    }
    if (ev & (EPOLLIN | EPOLLHUP | EPOLLERR)) {
      int r = slurp(epp_->fd, epp_->in);
      size_t off = 0;
      while (epp_->in.size() - off >= 4) {
        uint32_t n;
        memcpy(&n, epp_->in.data() + off, 4);
        n = ntohl(n);
        if (epp_->in.size() - off - 4 < n) break;
        Val msg;
        Up up{(const uint8_t*)epp_->in.data() + off + 4, (const uint8_t*)epp_->in.data() + off + 4 + n};
        up.read(msg);
        off += 4 + n;
        // An undecodable frame may have been a decision: its client would wait
        // in pending_ forever. Treat it as a lost EPP (fails every pick over).
        if (!up.ok) return epp_lost();
        on_epp_msg(msg);
        if (epp_ == nullptr) return;
      }
      epp_->in.erase(0, off);
      if (r <= 0) epp_lost();
    }
  }

  void on_epp_msg(const Val& msg) {
    const Val* eps = msg.get("eps");
    if (eps) {  // state reply
      eps_.clear();
      if (eps->t == Val::ARR)
        for (auto& e : eps->a) eps_.push_back(e.s);
      const Val* h = msg.get("health");
      if (h && h->t == Val::ARR && h->a.size() == 2) {
        health_status_ = (int)h->a[0].as_int(503);
        health_text_ = h->a[1].s;
      }
      const Val* c = msg.get("chunks");
      chunks_ = c && c->truthy();
      return;
    }
    const Val* id = msg.get("id");
    if (!id) return;
    auto pit = pending_.find((uint64_t)id->as_int());
    if (pit == pending_.end()) return;
    uint64_t cid = pit->second;
    pending_.erase(pit);
    auto cit = clients_.find(cid);
    const Val* d = msg.get("d");
    if (cit == clients_.end() || !cit->second->ex) {
      // the client went away while the EPP decided: release the decision
      if (d) send_done(d->get("tok") ? d->get("tok")->as_int() : 0, 499, -1, -1, 0, nullptr);
      return;
    }
    Client* c = cit->second;
    if (d) {
      Exchange& x = *c->ex;
      const Val* v;
      x.tok = (v = d->get("tok")) ? v->as_int() : 0;
      x.endpoint = (v = d->get("endpoint")) ? v->s : "";
      x.request_id = (v = d->get("request_id")) ? v->s : "";
      x.stream = (v = d->get("stream")) && v->truthy();
      if ((v = d->get("headers")) && v->t == Val::MAP)
        for (auto& kv : v->m) x.extra.emplace_back(kv.first, kv.second.s);
      if ((v = d->get("body")) && (v->t == Val::BIN || v->t == Val::STR)) {
        x.has_body_override = true;
        x.body_override = v->s;
      }
      forward(c);
      return;
    }
    const Val* err = msg.get("err");
    int st = err && err->get("status") ? (int)err->get("status")->as_int() : -1;
    std::string m = err && err->get("msg") ? err->get("msg")->s : "EPP error";
    if (st == -1) return epp_failed(c, m);
    std::string rsn = err && err->get("reason") ? err->get("reason")->s : "";
    Headers h;
    if (!rsn.empty()) h.emplace_back("x-llm-d-request-dropped-reason", rsn);
    respond_json(c, st, "{\"error\": {\"message\": " + json_str(m) + ", \"code\": " + std::to_string(st) + "}}", h);
  }

  void epp_failed(Client* c, const std::string& m) {
    if (!opt_.fail_open || eps_.empty()) {
      respond_json(c, 503, "{\"error\": {\"message\": " + json_str("endpoint picker failed: " + m) + "}}", {});
      return;
    }
    Exchange& x = *c->ex;
    x.tok = 0;  // fail-open: no EPP decision to complete
    x.endpoint = eps_[rng_() % eps_.size()];
    forward(c);
  }

  void send_done(int64_t tok, int status, double ttft, double tpot, double duration, const Val* usage) {
    if (tok <= 0) return;
    std::string m;
    Pk pk(m);
    pk.map(3);
    pk.str("op"); pk.str("done");
    pk.str("tok"); pk.integer(tok);
    pk.str("info");
    pk.map(4 + (tpot >= 0 ? 1 : 0));
    pk.str("status"); pk.integer(status);
    pk.str("duration"); pk.dbl(duration);
    pk.str("ttft");
    if (ttft >= 0) pk.dbl(ttft); else pk.nil();
    pk.str("usage");
    if (usage) pk.val(*usage); else pk.nil();
    if (tpot >= 0) { pk.str("tpot"); pk.dbl(tpot); }
    epp_send(m);
  }

  static std::string json_str(const std::string& s) {
    std::string o = "\"";
    for (char ch : s) {
      unsigned char u = (unsigned char)ch;
      if (ch == '"' || ch == '\\') { o.push_back('\\'); o.push_back(ch); }
      else if (u < 0x20) {
        char b[8];
        snprintf(b, sizeof b, "\\u%04x", u);
        o += b;
      } else o.push_back(ch);
    }
    return o + "\"";
  }

  // ---------------------------------------------------------------- clients
  void accept_all() {
    while (true) {
      int fd = accept4(lis_.fd, nullptr, nullptr, SOCK_NONBLOCK);
      if (fd < 0) return;
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      Client* c = new Client();
      c->kind = K_CLIENT;
      c->fd = fd;
      c->id = next_client_++;
      clients_[c->id] = c;
      add(c, EPOLLIN | EPOLLRDHUP);
    }
  }

  void client_events(Client* c) {
    if (c->dead) return;
    uint32_t ev = EPOLLRDHUP;
    if (!c->ex) ev |= EPOLLIN;  // one request at a time; the next waits in the socket
    if (!c->out.empty()) ev |= EPOLLOUT;
    mod(c, ev);
  }

  void client_close(Client* c) {
    if (c->dead) return;
    c->dead = true;
    if (c->ex) abort_exchange(c);
    clients_.erase(c->id);
    drop(c);
  }

  // the client is gone mid-exchange: release the upstream connection and the decision
  void abort_exchange(Client* c) {
    Exchange& x = *c->ex;
    if (x.up) {
      Upstream* u = x.up;
      x.up = nullptr;
      u->client = nullptr;
      drop(u);
      erase_connecting(u);
    }
    if (!x.finished) {
      x.finished = true;
      send_done(x.tok, x.status ? x.status : 499, x.first >= 0 ? x.first - x.t0 : -1, -1,
                x.t0 > 0 ? now_s() - x.t0 : 0, nullptr);
    }
    c->ex.reset();
  }

  void on_client(Client* c, uint32_t ev) {
    if (ev & EPOLLOUT) {
      if (!flush(c->fd, c->out, c->out_off)) return client_close(c);
      if (c->out.empty() && c->close_after && !c->ex) return client_close(c);
      // backpressure release: resume the upstream once the client drained
      if (c->ex && c->ex->up && c->out.size() - c->out_off < LOW_WATER) upstream_events(c->ex->up);
    }
    if (ev & EPOLLIN) {
      // EOF (or an error) ends the connection; a request still being relayed is released
      if (slurp(c->fd, c->in) <= 0) return client_close(c);
      if (!c->ex) try_request(c);
    } else if (ev & (EPOLLRDHUP | EPOLLHUP | EPOLLERR)) {
      // peer closed its side: if a response is still being relayed, the client is gone
      return client_close(c);
    }
    if (!c->dead) client_events(c);
  }

  // parse one complete request from c->in; false if malformed
  bool try_request(Client* c) {
    size_t he = c->in.find("\r\n\r\n");
    if (he == std::string::npos) {
      if (c->in.size() > (64u << 10)) { respond_simple_close(c, 431, "header too large"); return false; }
      return true;
    }
    const char* p = c->in.data();
    const char* le = (const char*)memchr(p, '\n', he + 2);
    std::string rl(p, le - p);
    if (!rl.empty() && rl.back() == '\r') rl.pop_back();
    size_t s1 = rl.find(' '), s2 = rl.rfind(' ');
    if (s1 == std::string::npos || s2 == s1) { respond_simple_close(c, 400, "bad request line"); return false; }
    auto x = std::make_unique<Exchange>();
    x->method = rl.substr(0, s1);
    x->target = rl.substr(s1 + 1, s2 - s1 - 1);
    std::string ver = rl.substr(s2 + 1);
    if (!parse_headers(le + 1, p + he + 2, x->hdrs)) { respond_simple_close(c, 400, "bad header"); return false; }
    size_t q = x->target.find('?');
    x->path = q == std::string::npos ? x->target : x->target.substr(0, q);
    const std::string* conn = hget(x->hdrs, "connection");
    x->keep_alive = ver == "HTTP/1.1" ? !(conn && ieq(*conn, "close")) : (conn && ieq(*conn, "keep-alive"));
    size_t body_at = he + 4;
    const std::string* te = hget(x->hdrs, "transfer-encoding");
    if (te && lower(*te).find("chunked") != std::string::npos) {
      long used = c->req_ck.feed(c->in.data() + body_at + c->req_fed, c->in.data() + c->in.size(),
                                 [&](const char* d, size_t n) { c->req_body.append(d, n); });
      if (used < 0) { respond_simple_close(c, 400, "bad chunked body"); return false; }
      c->req_fed += (size_t)used;
      // the same 256 MB cap as a Content-Length body, on the decoded body and
      // on what is buffered (chunk-size lines and extensions count too)
      // (a declared chunk size that would pass it is refused at once)
      if (c->req_body.size() + c->req_ck.left > (256u << 20) || c->req_fed > (256u << 20) + (1u << 20)) {
        respond_simple_close(c, 413, "body too large");
        return false;
      }
      if (c->req_ck.st != Chunked::DONE) return true;  // wait for the rest
      x->body = std::move(c->req_body);
      c->in.erase(0, body_at + c->req_fed);
      c->req_ck = Chunked();
      c->req_body.clear();
      c->req_fed = 0;
    } else {
      const std::string* cl = hget(x->hdrs, "content-length");
      size_t n = cl ? strtoull(cl->c_str(), nullptr, 10) : 0;
      if (n > (256u << 20)) { respond_simple_close(c, 413, "body too large"); return false; }
      if (c->in.size() - body_at < n) {
        const std::string* ex = hget(x->hdrs, "expect");
        if (ex && ieq(*ex, "100-continue") && !c->sent_continue) {
          c->sent_continue = true;
          c->out += "HTTP/1.1 100 Continue\r\n\r\n";
          if (!flush(c->fd, c->out, c->out_off)) { client_close(c); return false; }
        }
        return true;
      }
      x->body = c->in.substr(body_at, n);
      c->in.erase(0, body_at + n);
    }
    c->sent_continue = false;
    c->ex = std::move(x);
    handle(c);
    return true;
  }

  void handle(Client* c) {
    Exchange& x = *c->ex;
    if (x.path == "/health" && x.method == "GET") {
      return respond(c, health_status_, "text/plain; charset=utf-8", health_text_, {});
    }
    if (x.path == "/metrics") return respond(c, 200, "text/plain; charset=utf-8", "", {});
    if (health_text_ == "standby") {
      return respond_json(c, 503, "{\"error\": {\"message\": \"endpoint picker standby (not the HA leader)\"}}",
                          {{"x-llm-d-epp-role", "standby"}});
    }
    x.inference = x.method == "POST" && inference_path(x.path);
    if (!x.inference) {
      if (eps_.empty()) return respond_json(c, 503, "{\"error\": {\"message\": \"no endpoints\"}}", {});
      x.endpoint = eps_[rng_() % eps_.size()];
      return forward(c);
    }
    if (epp_ == nullptr) return epp_failed(c, "EPP connection lost");
    uint64_t id = next_id_++;
    pending_[id] = c->id;
    std::string m;
    Pk pk(m);
    pk.map(5);
    pk.str("op"); pk.str("pick");
    pk.str("id"); pk.integer((int64_t)id);
    pk.str("path"); pk.str(x.path);
    pk.str("headers");
    pk.map(x.hdrs.size());
    for (auto& kv : x.hdrs) { pk.str(kv.first); pk.str(kv.second); }
    pk.str("body"); pk.bin(x.body.data(), x.body.size());
    epp_send(m);
  }

  void respond(Client* c, int st, const char* ctype, const std::string& body, const Headers& extra) {
    std::string& o = c->out;
    o += "HTTP/1.1 " + std::to_string(st) + " " + reason(st) + "\r\nContent-Type: " + ctype +
         "\r\nContent-Length: " + std::to_string(body.size()) + "\r\n";
    for (auto& kv : extra) o += kv.first + ": " + kv.second + "\r\n";
    bool keep = c->ex ? c->ex->keep_alive : false;
    if (!keep) o += "Connection: close\r\n";
    o += "\r\n";
    o += body;
    finish_client(c, keep);
  }
  void respond_json(Client* c, int st, const std::string& body, const Headers& extra) {
    respond(c, st, "application/json; charset=utf-8", body, extra);
  }
  void respond_simple_close(Client* c, int st, const char* msg) {
    c->ex.reset();
    respond(c, st, "text/plain; charset=utf-8", msg, {});
  }

  // the exchange is over (response fully queued): next request or close after the flush
  void finish_client(Client* c, bool keep) {
    c->ex.reset();
    if (!keep) c->close_after = true;
    if (!flush(c->fd, c->out, c->out_off)) return client_close(c);
    if (c->close_after && c->out.empty()) return client_close(c);
    if (!c->close_after && !c->in.empty()) {
      if (!try_request(c)) return;
      if (c->dead) return;
    }
    client_events(c);
  }

  // ---------------------------------------------------------------- upstreams
  bool resolve(const std::string& key, sockaddr_storage& out, socklen_t& len) {
    auto it = addr_cache_.find(key);
    if (it != addr_cache_.end()) {
      out = it->second;
      len = out.ss_family == AF_INET6 ? sizeof(sockaddr_in6) : sizeof(sockaddr_in);
      return true;
    }
    size_t colon = key.rfind(':');
    if (colon == std::string::npos) return false;
    std::string host = key.substr(0, colon), port = key.substr(colon + 1);
    if (host.size() > 2 && host.front() == '[' && host.back() == ']') host = host.substr(1, host.size() - 2);
    addrinfo hints{}, *res = nullptr;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host.c_str(), port.c_str(), &hints, &res) != 0 || !res) return false;
    memcpy(&out, res->ai_addr, res->ai_addrlen);
    len = res->ai_addrlen;
    freeaddrinfo(res);
    addr_cache_[key] = out;
    return true;
  }

  Upstream* get_upstream(const std::string& key, bool allow_pool) {
    if (allow_pool) {
      auto& v = pool_[key];
      while (!v.empty()) {
        Upstream* u = v.back();
        v.pop_back();
        if (u->fd >= 0) {
          u->reused = true;
          return u;
        }
      }
    }
    sockaddr_storage sa;
    socklen_t len;
    if (!resolve(key, sa, len)) return nullptr;
    int fd = socket(sa.ss_family, SOCK_STREAM | SOCK_NONBLOCK, 0);
    if (fd < 0) return nullptr;
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    int r = connect(fd, (sockaddr*)&sa, len);
    if (r < 0 && errno != EINPROGRESS) {
      close(fd);
      return nullptr;
    }
    Upstream* u = new Upstream();
    u->kind = K_UP;
    u->fd = fd;
    u->key = key;
    u->connecting = r < 0;
    u->t_conn = now_s();
    add(u, EPOLLOUT | EPOLLRDHUP);
    if (u->connecting) connecting_.push_back(u);
    return u;
  }

  void erase_connecting(Upstream* u) {
    for (size_t k = 0; k < connecting_.size(); ++k)
      if (connecting_[k] == u) {
        connecting_[k] = connecting_.back();
        connecting_.pop_back();
        return;
      }
  }

  void check_connect_timeouts(double t) {
    for (size_t k = 0; k < connecting_.size();) {
      Upstream* u = connecting_[k];
      if (t - u->t_conn > 5.0) {
        connecting_[k] = connecting_.back();
        connecting_.pop_back();
        upstream_failed(u, "connect timeout");
      } else {
        ++k;
      }
    }
  }

  void upstream_events(Upstream* u) {
    if (u->fd < 0) return;
    uint32_t ev = EPOLLRDHUP;
    if (u->connecting || !u->out.empty()) ev |= EPOLLOUT;
    if (!u->connecting) {
      bool paused = u->client && u->client->out.size() - u->client->out_off >= HIGH_WATER;
      if (!paused) ev |= EPOLLIN;
    }
    mod(u, ev);
  }

  static std::string traceparent(const Headers& h, std::mt19937_64& rng) {
    char span[17];
    snprintf(span, sizeof span, "%016llx", (unsigned long long)rng());
    const std::string* tp = hget(h, "traceparent");
    if (tp && tp->size() >= 55 && (*tp)[2] == '-' && (*tp)[35] == '-' && (*tp)[52] == '-')
      return tp->substr(0, 36) + span + tp->substr(52);
    char trace[33];
    snprintf(trace, sizeof trace, "%016llx%016llx", (unsigned long long)rng(), (unsigned long long)rng());
    return std::string("00-") + trace + "-" + span + "-01";
  }

  void forward(Client* c) {
    Exchange& x = *c->ex;
    Upstream* u = get_upstream(x.endpoint, !x.retried);
    x.t0 = x.t0 > 0 ? x.t0 : now_s();
    if (u == nullptr) return upstream_error(c, "connect failed");
    u->client = c;
    x.up = u;
    // request: client headers minus hop-by-hop, then the decision's headers (they win), request id, trace
    const std::string& body = x.has_body_override ? x.body_override : x.body;
    std::string& o = u->out;
    o.clear();
    u->out_off = 0;
    o += (x.inference ? x.method + " " + x.path : x.method + " " + x.target) + " HTTP/1.1\r\nHost: " + x.endpoint + "\r\n";
    for (auto& kv : x.hdrs) {
      if (hop_header(kv.first) || ieq(kv.first, "traceparent") || ieq(kv.first, "expect")) continue;
      if (x.inference) {
        bool over = ieq(kv.first, "x-request-id");
        for (auto& e : x.extra) over = over || ieq(kv.first, e.first.c_str());
        if (over) continue;
      }
      o += kv.first + ": " + kv.second + "\r\n";
    }
    if (x.inference) {
      for (auto& e : x.extra) o += e.first + ": " + e.second + "\r\n";
      if (!x.request_id.empty()) o += "x-request-id: " + x.request_id + "\r\n";
    }
    o += "traceparent: " + traceparent(x.hdrs, rng_) + "\r\n";
    if (!body.empty() || x.method == "POST" || x.method == "PUT" || x.method == "PATCH")
      o += "Content-Length: " + std::to_string(body.size()) + "\r\n";
    o += "\r\n";
    o += body;
    if (!u->connecting) {
      if (!flush(u->fd, u->out, u->out_off)) return upstream_failed(u, "write failed");
    }
    upstream_events(u);
  }

  void upstream_error(Client* c, const std::string& why) {
    Exchange& x = *c->ex;
    x.finished = true;
    send_done(x.tok, 502, -1, -1, now_s() - x.t0, nullptr);
    respond_json(c, 502, "{\"error\": {\"message\": " + json_str("upstream " + x.endpoint + " failed: " + why) + "}}",
                 {});
  }

  // the upstream connection failed: retry once on a fresh connection if a pooled one died before
  // answering, else 502 (before the head) or abort the client stream (after it)
  void upstream_failed(Upstream* u, const char* why) {
    Client* c = u->client;
    u->client = nullptr;
    erase_connecting(u);
    drop(u);
    if (c == nullptr || !c->ex) return;
    Exchange& x = *c->ex;
    x.up = nullptr;
    if (!x.head_sent) {
      if (u->reused && !u->got_bytes && !x.retried) {
        x.retried = true;
        return forward(c);
      }
      return upstream_error(c, why);
    }
    x.finished = true;
    send_done(x.tok, x.status, x.first >= 0 ? x.first - x.t0 : -1, -1, now_s() - x.t0, nullptr);
    c->ex.reset();
    c->close_after = true;
    if (!flush(c->fd, c->out, c->out_off) || c->out.empty()) return client_close(c);
    client_events(c);
  }

  void on_upstream(Upstream* u, uint32_t ev) {
    if (u->client == nullptr) {  // idle in the pool: the server closed it (or sent junk)
      for (auto& kv : pool_) {
        auto& v = kv.second;
        for (size_t k = 0; k < v.size(); ++k)
          if (v[k] == u) {
            v[k] = v.back();
            v.pop_back();
            break;
          }
      }
      drop(u);
      return;
    }
    if (u->connecting && (ev & (EPOLLOUT | EPOLLERR | EPOLLHUP))) {
      int err = 0;
      socklen_t l = sizeof err;
      getsockopt(u->fd, SOL_SOCKET, SO_ERROR, &err, &l);
      if (err != 0) return upstream_failed(u, strerror(err));
      u->connecting = false;
      erase_connecting(u);
    }
    if (ev & EPOLLOUT) {
      if (!flush(u->fd, u->out, u->out_off)) return upstream_failed(u, "write failed");
    }
    if (ev & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) {
      int r = slurp(u->fd, u->in);
      if (!u->in.empty()) u->got_bytes = true;
      if (r < 0 && u->in.empty()) return upstream_failed(u, "connection reset");
      if (!process_response(u, r <= 0)) return;
      if (r <= 0) {
        if (u->client) return upstream_failed(u, "connection closed");
        return;
      }
    }
    upstream_events(u);
  }

  // relay what arrived; returns false if u was released (exchange finished or failed)
  bool process_response(Upstream* u, bool eof) {
    Client* c = u->client;
    Exchange& x = *c->ex;
    if (!x.head_sent) {
      size_t he = u->in.find("\r\n\r\n");
      if (he == std::string::npos) {
        if (u->in.size() > (64u << 10)) { upstream_failed(u, "response head too large"); return false; }
        return true;
      }
      const char* p = u->in.data();
      const char* le = (const char*)memchr(p, '\n', he + 2);
      std::string sl(p, le - p);
      if (sl.size() < 12 || sl.compare(0, 5, "HTTP/") != 0) { upstream_failed(u, "bad status line"); return false; }
      x.status = atoi(sl.c_str() + 9);
      bool up11 = sl.compare(0, 8, "HTTP/1.1") == 0;
      Headers rh;
      parse_headers(le + 1, p + he + 2, rh);
      u->in.erase(0, he + 4);
      if (x.status >= 100 && x.status < 200) return process_response(u, eof);  // interim response: skip
      const std::string* te = hget(rh, "transfer-encoding");
      const std::string* cl = hget(rh, "content-length");
      const std::string* conn = hget(rh, "connection");
      x.up_keep = up11 ? !(conn && ieq(*conn, "close")) : (conn && ieq(*conn, "keep-alive"));
      bool nobody = x.method == "HEAD" || x.status == 204 || x.status == 304 || (x.status >= 100 && x.status < 200);
      if (nobody) { x.framing = Exchange::F_LEN; x.remaining = 0; }
      else if (te && lower(*te).find("chunked") != std::string::npos) x.framing = Exchange::F_CHUNKED;
      else if (cl) { x.framing = Exchange::F_LEN; x.remaining = strtoull(cl->c_str(), nullptr, 10); }
      else { x.framing = Exchange::F_CLOSE; x.up_keep = false; }
      if (x.tok > 0) {  // response headers -> the EPP's response-header hooks
        std::string m;
        Pk pk(m);
        size_t nh = 0;
        for (auto& kv : rh) nh += !hop_header(kv.first);
        pk.map(4);
        pk.str("op"); pk.str("hdr");
        pk.str("tok"); pk.integer(x.tok);
        pk.str("status"); pk.integer(x.status);
        pk.str("headers");
        pk.map(nh);
        for (auto& kv : rh)
          if (!hop_header(kv.first)) { pk.str(kv.first); pk.str(kv.second); }
        epp_send(m);
      }
      std::string& o = c->out;
      o += "HTTP/1.1 " + std::to_string(x.status) + " " + reason(x.status) + "\r\n";
      for (auto& kv : rh)
        if (!hop_header(kv.first)) o += kv.first + ": " + kv.second + "\r\n";
      if (x.framing == Exchange::F_CHUNKED || x.framing == Exchange::F_CLOSE) {
        o += "Transfer-Encoding: chunked\r\n";
        x.rechunk = x.framing == Exchange::F_CLOSE;
      } else {
        o += "Content-Length: " + std::to_string(x.remaining) + "\r\n";
      }
      if (!x.keep_alive) o += "Connection: close\r\n";
      o += "\r\n";
      x.head_sent = true;
    }
    // body
    size_t take = 0;
    bool done = false;
    auto payload = [&](const char* d, size_t n) {
      if (n == 0) return;
      double t = now_s();
      if (x.first < 0) x.first = t;
      x.last = t;
      x.tail.append(d, n);
      if (x.tail.size() > 131072) x.tail.erase(0, x.tail.size() - 65536);
      if (chunks_ && x.tok > 0) {
        std::string m;
        Pk pk(m);
        pk.map(4);
        pk.str("op"); pk.str("chunk");
        pk.str("tok"); pk.integer(x.tok);
        pk.str("chunk"); pk.bin(d, n);
        pk.str("t"); pk.dbl(t);
        epp_send(m);
      }
    };
    if (x.framing == Exchange::F_LEN) {
      take = (size_t)std::min<uint64_t>(x.remaining, u->in.size());
      payload(u->in.data(), take);
      x.remaining -= take;
      c->out.append(u->in, 0, take);
      done = x.remaining == 0;
    } else if (x.framing == Exchange::F_CHUNKED) {
      long used = x.chunked.feed(u->in.data(), u->in.data() + u->in.size(), payload);
      if (used < 0) { upstream_failed(u, "bad chunked response"); return false; }
      take = (size_t)used;
      c->out.append(u->in, 0, take);  // verbatim: the client gets the upstream's own chunk framing
      done = x.chunked.st == Chunked::DONE;
    } else {  // close-delimited: re-framed as chunks
      take = u->in.size();
      if (take) {
        payload(u->in.data(), take);
        char sz[24];
        snprintf(sz, sizeof sz, "%zx\r\n", take);
        c->out += sz;
        c->out.append(u->in, 0, take);
        c->out += "\r\n";
      }
      if (eof) {
        c->out += "0\r\n\r\n";
        done = true;
      }
    }
    u->in.erase(0, take);
    if (!flush(c->fd, c->out, c->out_off)) {
      client_close(c);  // releases u too
      return false;
    }
    if (!done) return true;
    // exchange complete
    double end = now_s();
    x.finished = true;
    Val usage;
    bool have_usage = find_usage(x.tail, usage);
    double ttft = (x.first >= 0 && (x.stream || x.status == 200)) ? x.first - x.t0 : -1;
    double tpot = -1;
    if (have_usage && x.first >= 0) {
      const Val* n = usage.get("completion_tokens");
      int64_t k = n ? n->as_int() : 0;
      if (k > 1) tpot = (x.last - x.first) / (double)(k - 1);
    }
    send_done(x.tok, x.status, ttft, tpot, end - x.t0, have_usage ? &usage : nullptr);
    x.up = nullptr;
    u->client = nullptr;
    u->in.clear();
    if (x.up_keep && !eof && u->fd >= 0) {
      u->reused = false;
      u->got_bytes = false;
      pool_[u->key].push_back(u);
      mod(u, EPOLLIN | EPOLLRDHUP);  // an idle close / junk shows up as readable -> dropped
    } else {
      drop(u);
    }
    finish_client(c, x.keep_alive);
    return false;
  }
};

}  // namespace

int main(int argc, char** argv) {
  signal(SIGPIPE, SIG_IGN);
  Options o;
  for (int k = 1; k < argc; ++k) {
    std::string a = argv[k];
    auto next = [&]() -> std::string {
      if (k + 1 >= argc) {
        fprintf(stderr, "llmd-relay: %s needs a value\n", a.c_str());
        exit(2);
      }
      return argv[++k];
    };
    if (a == "--port") o.port = atoi(next().c_str());
    else if (a == "--uds") o.uds = next();
    else if (a == "--host") o.host = next();
    else if (a == "--threads") o.threads = atoi(next().c_str());
    else if (a == "--failure-mode") o.fail_open = next() == "FailOpen";
    else {
      fprintf(stderr, "usage: llmd-relay --port P --uds PATH [--host H] [--threads N] [--failure-mode M]\n");
      return 2;
    }
  }
  if (o.port <= 0 || o.uds.empty() || o.threads < 1) {
    fprintf(stderr, "llmd-relay: --port and --uds are required\n");
    return 2;
  }
  std::atomic<int> rc{0};
  std::vector<std::thread> th;
  for (int i = 0; i < o.threads; ++i)
    th.emplace_back([&, i] {
      Loop l(o, i);
      int r = l.run();
      rc = r;
      exit(r);  // a thread that cannot serve takes the process down; the parent restarts it
    });
  fprintf(stderr, "llmd-relay: %d threads on %s:%d (EPP %s)\n", o.threads, o.host.c_str(), o.port, o.uds.c_str());
  for (auto& t : th) t.join();
  return rc;
}
