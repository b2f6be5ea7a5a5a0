// cloudtik-state-server: the head node's state service (native component N1).
//
// The reference vendors and builds redis-server (build.sh:28-44) and uses a subset of its
// command set for the control plane's KV namespaces, node / process / metrics tables and
// log / error pub-sub (core/_private/state/redis_shards_client.py:36-140,
// control_state.py:37-151).  This is a purpose-built replacement: a single-threaded epoll
// server speaking RESP2 with exactly that subset, plus snapshot persistence:
//
//   PING ECHO AUTH SELECT QUIT
//   GET SET(NX|XX|EX|PX) SETNX DEL EXISTS MGET MSET KEYS SCAN INCR INCRBY EXPIRE TTL TYPE
//   RPUSH LPUSH LRANGE LLEN LPOP RPOP LTRIM
//   HSET HGET HDEL HGETALL HKEYS HLEN HEXISTS HINCRBY
//   PUBLISH SUBSCRIBE UNSUBSCRIBE PSUBSCRIBE PUNSUBSCRIBE
//   CONFIG GET|SET  CLIENT LIST|SETNAME  DBSIZE FLUSHALL FLUSHDB SAVE BGSAVE LASTSAVE INFO
//   SHUTDOWN
//
// Usage: cloudtik-state-server [--port N] [--bind ADDR] [--requirepass PW] [--dir D]
//                              [--dbfilename F] [--save-interval S]
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fnmatch.h>
#include <fstream>
#include <map>
#include <memory>
#include <set>
#include <sstream>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {

using Clock = std::chrono::steady_clock;

int64_t now_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::system_clock::now().time_since_epoch()).count();
}

enum class VT { STR, LIST, HASH };

struct Value {
  VT type = VT::STR;
  std::string str;
  std::deque<std::string> list;
  std::unordered_map<std::string, std::string> hash;
  int64_t expire_ms = -1;  // absolute unix ms, -1 = none
};

struct Client {
  int fd;
  uint64_t id;
  std::string in;
  std::string out;
  std::string name;
  std::string addr;
  bool authed = false;
  bool closing = false;
  std::set<std::string> channels, patterns;
  int64_t created_ms = 0;
};

struct Config {
  int port = 6789;
  std::string bind = "0.0.0.0";
  std::string password;
  std::string dir = ".";
  std::string dbfilename = "cloudtik-state.snapshot";
  int save_interval_s = 0;
  std::map<std::string, std::string> extra;  // CONFIG SET of unknown keys is remembered
};

Config g_cfg;
std::unordered_map<std::string, Value> g_db;
std::unordered_map<int, std::unique_ptr<Client>> g_clients;
std::unordered_map<std::string, std::unordered_set<int>> g_channels;
std::unordered_map<std::string, std::unordered_set<int>> g_patterns;
uint64_t g_next_id = 1;
int64_t g_lastsave = 0;
uint64_t g_dirty = 0;
int g_epfd = -1;
volatile sig_atomic_t g_stop = 0;

// ------------------------------------------------------------------ RESP encoding
void w_simple(Client& c, const std::string& s) { c.out += "+" + s + "\r\n"; }
void w_err(Client& c, const std::string& s) { c.out += "-ERR " + s + "\r\n"; }
void w_int(Client& c, long long v) { c.out += ":" + std::to_string(v) + "\r\n"; }
void w_bulk(Client& c, const std::string& s) {
  c.out += "$" + std::to_string(s.size()) + "\r\n";
  c.out += s;
  c.out += "\r\n";
}
void w_nil(Client& c) { c.out += "$-1\r\n"; }
void w_arr(Client& c, size_t n) { c.out += "*" + std::to_string(n) + "\r\n"; }

std::string upper(std::string s) {
  for (auto& ch : s) ch = (char)toupper((unsigned char)ch);
  return s;
}

// ------------------------------------------------------------------ keyspace helpers
Value* lookup(const std::string& k) {
  auto it = g_db.find(k);
  if (it == g_db.end()) return nullptr;
  if (it->second.expire_ms >= 0 && it->second.expire_ms <= now_ms()) {
    g_db.erase(it);
    return nullptr;
  }
  return &it->second;
}

bool wrongtype(Client& c, Value* v, VT t) {
  if (v && v->type != t) {
    c.out += "-WRONGTYPE Operation against a key holding the wrong kind of value\r\n";
    return true;
  }
  return false;
}

bool parse_ll(const std::string& s, long long& out) {
  char* e = nullptr;
  errno = 0;
  out = strtoll(s.c_str(), &e, 10);
  return errno == 0 && e && *e == 0 && !s.empty();
}

// ------------------------------------------------------------------ persistence
// snapshot format: "CTSS1\n" then records  <type> <len>:<key> ... with length-prefixed strings
void put_str(std::ostream& o, const std::string& s) { o << s.size() << ':' << s; }
bool get_str(std::istream& i, std::string& s) {
  size_t n;
  char colon;
  if (!(i >> n)) return false;
  if (!i.get(colon) || colon != ':') return false;
  s.resize(n);
  return (bool)i.read(&s[0], (std::streamsize)n) || n == 0;
}

bool save_snapshot() {
  const std::string path = g_cfg.dir + "/" + g_cfg.dbfilename;
  const std::string tmp = path + ".tmp";
  std::ofstream o(tmp, std::ios::binary | std::ios::trunc);
  if (!o) return false;
  o << "CTSS1\n";
  const int64_t t = now_ms();
  for (auto& kv : g_db) {
    const Value& v = kv.second;
    if (v.expire_ms >= 0 && v.expire_ms <= t) continue;
    o << (v.type == VT::STR ? 'S' : v.type == VT::LIST ? 'L' : 'H') << ' ' << v.expire_ms << ' ';
    put_str(o, kv.first);
    if (v.type == VT::STR) {
      put_str(o, v.str);
    } else if (v.type == VT::LIST) {
      o << v.list.size() << ' ';
      for (auto& e : v.list) put_str(o, e);
    } else {
      o << v.hash.size() << ' ';
      for (auto& e : v.hash) { put_str(o, e.first); put_str(o, e.second); }
    }
    o << '\n';
  }
  o.close();
  if (!o) return false;
  if (rename(tmp.c_str(), path.c_str()) != 0) return false;
  g_lastsave = now_ms() / 1000;
  g_dirty = 0;
  return true;
}

void load_snapshot() {
  const std::string path = g_cfg.dir + "/" + g_cfg.dbfilename;
  std::ifstream i(path, std::ios::binary);
  if (!i) return;
  std::string magic;
  std::getline(i, magic);
  if (magic != "CTSS1") return;
  char type;
  while (i >> type) {
    Value v;
    long long exp;
    i >> exp;
    v.expire_ms = exp;
    i.get();
    std::string key;
    if (!get_str(i, key)) break;
    if (type == 'S') {
      v.type = VT::STR;
      if (!get_str(i, v.str)) break;
    } else if (type == 'L') {
      v.type = VT::LIST;
      size_t n;
      i >> n;
      i.get();
      for (size_t k = 0; k < n; ++k) { std::string e; get_str(i, e); v.list.push_back(e); }
    } else {
      v.type = VT::HASH;
      size_t n;
      i >> n;
      i.get();
      for (size_t k = 0; k < n; ++k) { std::string a, b; get_str(i, a); get_str(i, b); v.hash[a] = b; }
    }
    g_db[key] = std::move(v);
  }
}

// ------------------------------------------------------------------ pub/sub
size_t publish(const std::string& ch, const std::string& msg) {
  size_t n = 0;
  auto it = g_channels.find(ch);
  if (it != g_channels.end()) {
    for (int fd : it->second) {
      auto c = g_clients.find(fd);
      if (c == g_clients.end()) continue;
      w_arr(*c->second, 3); w_bulk(*c->second, "message"); w_bulk(*c->second, ch); w_bulk(*c->second, msg);
      ++n;
    }
  }
  for (auto& p : g_patterns) {
    if (fnmatch(p.first.c_str(), ch.c_str(), 0) != 0) continue;
    for (int fd : p.second) {
      auto c = g_clients.find(fd);
      if (c == g_clients.end()) continue;
      w_arr(*c->second, 4); w_bulk(*c->second, "pmessage"); w_bulk(*c->second, p.first);
      w_bulk(*c->second, ch); w_bulk(*c->second, msg);
      ++n;
    }
  }
  return n;
}

void unsubscribe_all(Client& c) {
  for (auto& ch : c.channels) {
    auto it = g_channels.find(ch);
    if (it != g_channels.end()) { it->second.erase(c.fd); if (it->second.empty()) g_channels.erase(it); }
  }
  for (auto& p : c.patterns) {
    auto it = g_patterns.find(p);
    if (it != g_patterns.end()) { it->second.erase(c.fd); if (it->second.empty()) g_patterns.erase(it); }
  }
  c.channels.clear();
  c.patterns.clear();
}

// ------------------------------------------------------------------ command dispatch
void cmd(Client& c, std::vector<std::string>& a) {
  if (a.empty()) return;
  const std::string op = upper(a[0]);
  const size_t n = a.size();
  auto arity = [&](size_t lo, size_t hi = 1u << 30) {
    if (n < lo || n > hi) { w_err(c, "wrong number of arguments for '" + a[0] + "' command"); return false; }
    return true;
  };
  if (op == "AUTH") {
    if (!arity(2, 3)) return;
    if (g_cfg.password.empty() || a.back() == g_cfg.password) { c.authed = true; w_simple(c, "OK"); }
    else c.out += "-WRONGPASS invalid password\r\n";
    return;
  }
  if (!g_cfg.password.empty() && !c.authed && op != "PING" && op != "QUIT") {
    c.out += "-NOAUTH Authentication required.\r\n";
    return;
  }
  if (op == "PING") { if (n > 1) w_bulk(c, a[1]); else w_simple(c, "PONG"); return; }
  if (op == "ECHO") { if (arity(2, 2)) w_bulk(c, a[1]); return; }
  if (op == "QUIT") { w_simple(c, "OK"); c.closing = true; return; }
  if (op == "SELECT") { w_simple(c, "OK"); return; }
  if (op == "GET") {
    if (!arity(2, 2)) return;
    Value* v = lookup(a[1]);
    if (wrongtype(c, v, VT::STR)) return;
    if (v) w_bulk(c, v->str); else w_nil(c);
    return;
  }
  if (op == "SET") {
    if (!arity(3)) return;
    bool nx = false, xx = false;
    int64_t exp = -1;
    for (size_t i = 3; i < n; ++i) {
      const std::string o = upper(a[i]);
      long long t;
      if (o == "NX") nx = true;
      else if (o == "XX") xx = true;
      else if ((o == "EX" || o == "PX") && i + 1 < n && parse_ll(a[i + 1], t)) {
        exp = now_ms() + (o == "EX" ? t * 1000 : t);
        ++i;
      } else { w_err(c, "syntax error"); return; }
    }
    Value* cur = lookup(a[1]);
    if ((nx && cur) || (xx && !cur)) { w_nil(c); return; }
    Value v;
    v.type = VT::STR;
    v.str = a[2];
    v.expire_ms = exp;
    g_db[a[1]] = std::move(v);
    ++g_dirty;
    w_simple(c, "OK");
    return;
  }
  if (op == "SETNX") {
    if (!arity(3, 3)) return;
    if (lookup(a[1])) { w_int(c, 0); return; }
    Value v; v.str = a[2]; g_db[a[1]] = std::move(v); ++g_dirty; w_int(c, 1);
    return;
  }
  if (op == "MSET") {
    if (n < 3 || (n - 1) % 2) { w_err(c, "wrong number of arguments for 'mset' command"); return; }
    for (size_t i = 1; i + 1 < n; i += 2) { Value v; v.str = a[i + 1]; g_db[a[i]] = std::move(v); }
    ++g_dirty;
    w_simple(c, "OK");
    return;
  }
  if (op == "DEL" || op == "UNLINK") {
    if (!arity(2)) return;
    long long k = 0;
    for (size_t i = 1; i < n; ++i) if (lookup(a[i])) { g_db.erase(a[i]); ++k; }
    if (k) ++g_dirty;
    w_int(c, k);
    return;
  }
  if (op == "EXISTS") {
    if (!arity(2)) return;
    long long k = 0;
    for (size_t i = 1; i < n; ++i) if (lookup(a[i])) ++k;
    w_int(c, k);
    return;
  }
  if (op == "MGET") {
    if (!arity(2)) return;
    w_arr(c, n - 1);
    for (size_t i = 1; i < n; ++i) {
      Value* v = lookup(a[i]);
      if (v && v->type == VT::STR) w_bulk(c, v->str); else w_nil(c);
    }
    return;
  }
  if (op == "KEYS" || op == "SCAN") {
    std::string pat = "*";
    long long count = 1 << 30;
    size_t first = 1;
    if (op == "KEYS") { if (!arity(2, 2)) return; pat = a[1]; }
    else {
      if (!arity(2)) return;
      first = 2;
      for (size_t i = first; i + 1 < n; i += 2) {
        const std::string o = upper(a[i]);
        if (o == "MATCH") pat = a[i + 1];
        else if (o == "COUNT") parse_ll(a[i + 1], count);
      }
    }
    std::vector<std::string> out;
    const int64_t t = now_ms();
    for (auto& kv : g_db) {
      if (kv.second.expire_ms >= 0 && kv.second.expire_ms <= t) continue;
      if (fnmatch(pat.c_str(), kv.first.c_str(), 0) == 0) out.push_back(kv.first);
    }
    std::sort(out.begin(), out.end());
    if (op == "SCAN") { w_arr(c, 2); w_bulk(c, "0"); }   // single full-iteration cursor
    w_arr(c, out.size());
    for (auto& k : out) w_bulk(c, k);
    return;
  }
  if (op == "INCR" || op == "INCRBY" || op == "DECR") {
    if (!arity(op == "INCRBY" ? 3 : 2, op == "INCRBY" ? 3 : 2)) return;
    long long by = op == "DECR" ? -1 : 1;
    if (op == "INCRBY" && !parse_ll(a[2], by)) { w_err(c, "value is not an integer or out of range"); return; }
    Value* v = lookup(a[1]);
    if (wrongtype(c, v, VT::STR)) return;
    long long cur = 0;
    if (v && !parse_ll(v->str, cur)) { w_err(c, "value is not an integer or out of range"); return; }
    cur += by;
    Value& nv = g_db[a[1]];
    nv.type = VT::STR;
    nv.str = std::to_string(cur);
    ++g_dirty;
    w_int(c, cur);
    return;
  }
  if (op == "EXPIRE" || op == "PEXPIRE") {
    if (!arity(3, 3)) return;
    long long t;
    Value* v = lookup(a[1]);
    if (!v || !parse_ll(a[2], t)) { w_int(c, 0); return; }
    v->expire_ms = now_ms() + (op == "EXPIRE" ? t * 1000 : t);
    w_int(c, 1);
    return;
  }
  if (op == "TTL" || op == "PTTL") {
    if (!arity(2, 2)) return;
    Value* v = lookup(a[1]);
    if (!v) { w_int(c, -2); return; }
    if (v->expire_ms < 0) { w_int(c, -1); return; }
    const long long ms = v->expire_ms - now_ms();
    w_int(c, op == "TTL" ? ms / 1000 : ms);
    return;
  }
  if (op == "TYPE") {
    if (!arity(2, 2)) return;
    Value* v = lookup(a[1]);
    w_simple(c, !v ? "none" : v->type == VT::STR ? "string" : v->type == VT::LIST ? "list" : "hash");
    return;
  }
  // ---- lists
  if (op == "RPUSH" || op == "LPUSH") {
    if (!arity(3)) return;
    Value* v = lookup(a[1]);
    if (wrongtype(c, v, VT::LIST)) return;
    Value& L = g_db[a[1]];
    L.type = VT::LIST;
    for (size_t i = 2; i < n; ++i) {
      if (op == "RPUSH") L.list.push_back(a[i]); else L.list.push_front(a[i]);
    }
    ++g_dirty;
    w_int(c, (long long)L.list.size());
    return;
  }
  if (op == "LRANGE") {
    if (!arity(4, 4)) return;
    Value* v = lookup(a[1]);
    if (wrongtype(c, v, VT::LIST)) return;
    long long s, e;
    if (!parse_ll(a[2], s) || !parse_ll(a[3], e)) { w_err(c, "value is not an integer"); return; }
    if (!v) { w_arr(c, 0); return; }
    const long long len = (long long)v->list.size();
    if (s < 0) s += len;
    if (e < 0) e += len;
    s = std::max(0LL, s);
    e = std::min(len - 1, e);
    if (s > e) { w_arr(c, 0); return; }
    w_arr(c, (size_t)(e - s + 1));
    for (long long i = s; i <= e; ++i) w_bulk(c, v->list[(size_t)i]);
    return;
  }
  if (op == "LLEN") {
    if (!arity(2, 2)) return;
    Value* v = lookup(a[1]);
    if (wrongtype(c, v, VT::LIST)) return;
    w_int(c, v ? (long long)v->list.size() : 0);
    return;
  }
  if (op == "LPOP" || op == "RPOP") {
    if (!arity(2, 2)) return;
    Value* v = lookup(a[1]);
    if (wrongtype(c, v, VT::LIST)) return;
    if (!v || v->list.empty()) { w_nil(c); return; }
    std::string e;
    if (op == "LPOP") { e = v->list.front(); v->list.pop_front(); }
    else { e = v->list.back(); v->list.pop_back(); }
    if (v->list.empty()) g_db.erase(a[1]);
    ++g_dirty;
    w_bulk(c, e);
    return;
  }
  if (op == "LTRIM") {
    if (!arity(4, 4)) return;
    Value* v = lookup(a[1]);
    long long s, e;
    if (!v || !parse_ll(a[2], s) || !parse_ll(a[3], e)) { w_simple(c, "OK"); return; }
    const long long len = (long long)v->list.size();
    if (s < 0) s += len;
    if (e < 0) e += len;
    s = std::max(0LL, s);
    e = std::min(len - 1, e);
    std::deque<std::string> nl;
    for (long long i = s; i <= e; ++i) nl.push_back(v->list[(size_t)i]);
    v->list.swap(nl);
    ++g_dirty;
    w_simple(c, "OK");
    return;
  }
  // ---- hashes
  if (op == "HSET" || op == "HMSET") {
    if (n < 4 || (n - 2) % 2) { w_err(c, "wrong number of arguments for 'hset' command"); return; }
    Value* v = lookup(a[1]);
    if (wrongtype(c, v, VT::HASH)) return;
    Value& Hh = g_db[a[1]];
    Hh.type = VT::HASH;
    long long added = 0;
    for (size_t i = 2; i + 1 < n; i += 2) {
      if (!Hh.hash.count(a[i])) ++added;
      Hh.hash[a[i]] = a[i + 1];
    }
    ++g_dirty;
    if (op == "HMSET") w_simple(c, "OK"); else w_int(c, added);
    return;
  }
  if (op == "HGET") {
    if (!arity(3, 3)) return;
    Value* v = lookup(a[1]);
    if (wrongtype(c, v, VT::HASH)) return;
    if (!v) { w_nil(c); return; }
    auto it = v->hash.find(a[2]);
    if (it == v->hash.end()) w_nil(c); else w_bulk(c, it->second);
    return;
  }
  if (op == "HDEL") {
    if (!arity(3)) return;
    Value* v = lookup(a[1]);
    if (wrongtype(c, v, VT::HASH)) return;
    long long k = 0;
    if (v) for (size_t i = 2; i < n; ++i) k += (long long)v->hash.erase(a[i]);
    if (v && v->hash.empty()) g_db.erase(a[1]);
    if (k) ++g_dirty;
    w_int(c, k);
    return;
  }
  if (op == "HGETALL" || op == "HKEYS" || op == "HLEN") {
    if (!arity(2, 2)) return;
    Value* v = lookup(a[1]);
    if (wrongtype(c, v, VT::HASH)) return;
    if (op == "HLEN") { w_int(c, v ? (long long)v->hash.size() : 0); return; }
    std::vector<std::pair<std::string, std::string>> items;
    if (v) items.assign(v->hash.begin(), v->hash.end());
    std::sort(items.begin(), items.end());
    w_arr(c, op == "HGETALL" ? items.size() * 2 : items.size());
    for (auto& kv : items) { w_bulk(c, kv.first); if (op == "HGETALL") w_bulk(c, kv.second); }
    return;
  }
  if (op == "HEXISTS") {
    if (!arity(3, 3)) return;
    Value* v = lookup(a[1]);
    w_int(c, v && v->type == VT::HASH && v->hash.count(a[2]) ? 1 : 0);
    return;
  }
  if (op == "HINCRBY") {
    if (!arity(4, 4)) return;
    Value* v = lookup(a[1]);
    if (wrongtype(c, v, VT::HASH)) return;
    long long by, cur = 0;
    if (!parse_ll(a[3], by)) { w_err(c, "value is not an integer"); return; }
    Value& Hh = g_db[a[1]];
    Hh.type = VT::HASH;
    auto it = Hh.hash.find(a[2]);
    if (it != Hh.hash.end() && !parse_ll(it->second, cur)) { w_err(c, "hash value is not an integer"); return; }
    cur += by;
    Hh.hash[a[2]] = std::to_string(cur);
    ++g_dirty;
    w_int(c, cur);
    return;
  }
  // ---- lock primitives (atomic: the server is single-threaded)
  // DELIFEQ key token          -> 1 if key held token and was deleted (lock release)
  // PEXPIREIFEQ key token ms   -> 1 if key holds token and its TTL was reset (lease renewal)
  if (op == "DELIFEQ" || op == "PEXPIREIFEQ") {
    if (!arity(op == "DELIFEQ" ? 3 : 4, op == "DELIFEQ" ? 3 : 4)) return;
    Value* v = lookup(a[1]);
    if (!v || v->type != VT::STR || v->str != a[2]) { w_int(c, 0); return; }
    if (op == "DELIFEQ") {
      g_db.erase(a[1]);
    } else {
      long long ms;
      if (!parse_ll(a[3], ms)) { w_err(c, "value is not an integer"); return; }
      v->expire_ms = now_ms() + ms;
    }
    ++g_dirty;
    w_int(c, 1);
    return;
  }
  // ---- pub/sub
  if (op == "PUBLISH") {
    if (!arity(3, 3)) return;
    w_int(c, (long long)publish(a[1], a[2]));
    return;
  }
  if (op == "SUBSCRIBE" || op == "PSUBSCRIBE") {
    if (!arity(2)) return;
    const bool p = op == "PSUBSCRIBE";
    for (size_t i = 1; i < n; ++i) {
      (p ? c.patterns : c.channels).insert(a[i]);
      (p ? g_patterns : g_channels)[a[i]].insert(c.fd);
      w_arr(c, 3);
      w_bulk(c, p ? "psubscribe" : "subscribe");
      w_bulk(c, a[i]);
      w_int(c, (long long)(c.channels.size() + c.patterns.size()));
    }
    return;
  }
  if (op == "UNSUBSCRIBE" || op == "PUNSUBSCRIBE") {
    const bool p = op == "PUNSUBSCRIBE";
    std::vector<std::string> targets(a.begin() + 1, a.end());
    if (targets.empty()) targets.assign((p ? c.patterns : c.channels).begin(), (p ? c.patterns : c.channels).end());
    for (auto& t : targets) {
      (p ? c.patterns : c.channels).erase(t);
      auto& m = p ? g_patterns : g_channels;
      auto it = m.find(t);
      if (it != m.end()) { it->second.erase(c.fd); if (it->second.empty()) m.erase(it); }
      w_arr(c, 3);
      w_bulk(c, p ? "punsubscribe" : "unsubscribe");
      w_bulk(c, t);
      w_int(c, (long long)(c.channels.size() + c.patterns.size()));
    }
    return;
  }
  // ---- server
  if (op == "CONFIG") {
    if (!arity(3)) return;
    const std::string sub = upper(a[1]);
    if (sub == "GET") {
      std::vector<std::pair<std::string, std::string>> kv = {
          {"port", std::to_string(g_cfg.port)}, {"bind", g_cfg.bind}, {"dir", g_cfg.dir},
          {"dbfilename", g_cfg.dbfilename}, {"requirepass", g_cfg.password},
          {"save", std::to_string(g_cfg.save_interval_s)}};
      for (auto& e : g_cfg.extra) kv.push_back(e);
      std::vector<std::pair<std::string, std::string>> out;
      for (auto& e : kv) if (fnmatch(a[2].c_str(), e.first.c_str(), 0) == 0) out.push_back(e);
      w_arr(c, out.size() * 2);
      for (auto& e : out) { w_bulk(c, e.first); w_bulk(c, e.second); }
    } else if (sub == "SET") {
      if (!arity(4, 4)) return;
      const std::string k = a[2];
      if (k == "requirepass") g_cfg.password = a[3];
      else if (k == "dir") g_cfg.dir = a[3];
      else if (k == "dbfilename") g_cfg.dbfilename = a[3];
      else if (k == "save") g_cfg.save_interval_s = atoi(a[3].c_str());
      else g_cfg.extra[k] = a[3];
      w_simple(c, "OK");
    } else {
      w_err(c, "unknown CONFIG subcommand");
    }
    return;
  }
  if (op == "CLIENT") {
    if (!arity(2)) return;
    const std::string sub = upper(a[1]);
    if (sub == "LIST") {
      std::ostringstream o;
      const int64_t t = now_ms();
      for (auto& kv : g_clients) {
        const Client& x = *kv.second;
        o << "id=" << x.id << " addr=" << x.addr << " fd=" << x.fd << " name=" << x.name
          << " age=" << (t - x.created_ms) / 1000 << " sub=" << x.channels.size()
          << " psub=" << x.patterns.size() << "\n";
      }
      w_bulk(c, o.str());
    } else if (sub == "SETNAME" && n == 3) {
      c.name = a[2];
      w_simple(c, "OK");
    } else if (sub == "GETNAME") {
      w_bulk(c, c.name);
    } else if (sub == "ID") {
      w_int(c, (long long)c.id);
    } else {
      w_simple(c, "OK");
    }
    return;
  }
  if (op == "DBSIZE") { w_int(c, (long long)g_db.size()); return; }
  if (op == "FLUSHALL" || op == "FLUSHDB") { g_db.clear(); ++g_dirty; w_simple(c, "OK"); return; }
  if (op == "SAVE" || op == "BGSAVE") {
    if (save_snapshot()) w_simple(c, op == "SAVE" ? "OK" : "Background saving started");
    else w_err(c, "snapshot failed");
    return;
  }
  if (op == "LASTSAVE") { w_int(c, g_lastsave); return; }
  if (op == "INFO") {
    std::ostringstream o;
    o << "# Server\r\nserver:cloudtik-state-server\r\nversion:1.0\r\ntcp_port:" << g_cfg.port
      << "\r\nconnected_clients:" << g_clients.size() << "\r\n# Keyspace\r\ndb0:keys=" << g_db.size()
      << "\r\nchanges_since_last_save:" << g_dirty << "\r\n";
    w_bulk(c, o.str());
    return;
  }
  if (op == "SHUTDOWN") {
    if (n < 2 || upper(a[1]) != "NOSAVE") save_snapshot();
    g_stop = 1;
    w_simple(c, "OK");
    return;
  }
  w_err(c, "unknown command '" + a[0] + "'");
}

// ------------------------------------------------------------------ RESP parsing
// returns: 1 = parsed one command, 0 = need more data, -1 = protocol error
int parse_one(std::string& in, size_t& pos, std::vector<std::string>& out) {
  out.clear();
  if (pos >= in.size()) return 0;
  if (in[pos] != '*') {  // inline command
    size_t e = in.find("\r\n", pos);
    if (e == std::string::npos) return 0;
    std::istringstream ss(in.substr(pos, e - pos));
    std::string tok;
    while (ss >> tok) out.push_back(tok);
    pos = e + 2;
    return 1;
  }
  size_t e = in.find("\r\n", pos);
  if (e == std::string::npos) return 0;
  long long cnt;
  if (!parse_ll(in.substr(pos + 1, e - pos - 1), cnt) || cnt < 0 || cnt > (1 << 20)) return -1;
  size_t p = e + 2;
  for (long long i = 0; i < cnt; ++i) {
    if (p >= in.size()) return 0;
    if (in[p] != '$') return -1;
    size_t e2 = in.find("\r\n", p);
    if (e2 == std::string::npos) return 0;
    long long len;
    if (!parse_ll(in.substr(p + 1, e2 - p - 1), len) || len < 0 || len > (512LL << 20)) return -1;
    const size_t start = e2 + 2;
    if (in.size() < start + (size_t)len + 2) return 0;
    out.emplace_back(in, start, (size_t)len);
    p = start + (size_t)len + 2;
  }
  pos = p;
  return 1;
}

void set_nonblock(int fd) { fcntl(fd, F_SETFL, fcntl(fd, F_GETFL, 0) | O_NONBLOCK); }

void close_client(int fd) {
  auto it = g_clients.find(fd);
  if (it == g_clients.end()) return;
  unsubscribe_all(*it->second);
  epoll_ctl(g_epfd, EPOLL_CTL_DEL, fd, nullptr);
  close(fd);
  g_clients.erase(it);
}

void flush_client(Client& c) {
  while (!c.out.empty()) {
    ssize_t k = send(c.fd, c.out.data(), c.out.size(), MSG_NOSIGNAL);
    if (k > 0) { c.out.erase(0, (size_t)k); continue; }
    if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
    c.closing = true;
    c.out.clear();
    break;
  }
  epoll_event ev{};
  ev.events = EPOLLIN | (c.out.empty() ? 0 : EPOLLOUT);
  ev.data.fd = c.fd;
  epoll_ctl(g_epfd, EPOLL_CTL_MOD, c.fd, &ev);
}

void on_signal(int) { g_stop = 1; }

}  // namespace

int main(int argc, char** argv) {
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() { return i + 1 < argc ? std::string(argv[++i]) : std::string(); };
    if (a == "--port") g_cfg.port = atoi(next().c_str());
    else if (a == "--bind") g_cfg.bind = next();
    else if (a == "--requirepass") g_cfg.password = next();
    else if (a == "--dir") g_cfg.dir = next();
    else if (a == "--dbfilename") g_cfg.dbfilename = next();
    else if (a == "--save-interval") g_cfg.save_interval_s = atoi(next().c_str());
    else if (a == "--help" || a == "-h") {
      printf("usage: cloudtik-state-server [--port N] [--bind ADDR] [--requirepass PW] [--dir D] "
             "[--dbfilename F] [--save-interval S]\n");
      return 0;
    }
  }
  signal(SIGPIPE, SIG_IGN);
  signal(SIGTERM, on_signal);
  signal(SIGINT, on_signal);
  load_snapshot();

  const int lfd = socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons((uint16_t)g_cfg.port);
  if (inet_pton(AF_INET, g_cfg.bind.c_str(), &addr.sin_addr) != 1) addr.sin_addr.s_addr = INADDR_ANY;
  if (bind(lfd, (sockaddr*)&addr, sizeof(addr)) != 0 || listen(lfd, 512) != 0) {
    fprintf(stderr, "cloudtik-state-server: cannot listen on %s:%d: %s\n", g_cfg.bind.c_str(),
            g_cfg.port, strerror(errno));
    return 1;
  }
  set_nonblock(lfd);
  g_epfd = epoll_create1(0);
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = lfd;
  epoll_ctl(g_epfd, EPOLL_CTL_ADD, lfd, &ev);
  fprintf(stderr, "cloudtik-state-server listening on %s:%d\n", g_cfg.bind.c_str(), g_cfg.port);
  fflush(stderr);

  std::vector<epoll_event> events(256);
  auto last_save = Clock::now();
  std::vector<std::string> argvv;
  char buf[65536];
  while (!g_stop) {
    const int nev = epoll_wait(g_epfd, events.data(), (int)events.size(), 200);
    for (int e = 0; e < nev; ++e) {
      const int fd = events[e].data.fd;
      if (fd == lfd) {
        while (true) {
          sockaddr_in ca{};
          socklen_t cl = sizeof(ca);
          const int cfd = accept(lfd, (sockaddr*)&ca, &cl);
          if (cfd < 0) break;
          set_nonblock(cfd);
          setsockopt(cfd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
          auto c = std::make_unique<Client>();
          c->fd = cfd;
          c->id = g_next_id++;
          c->created_ms = now_ms();
          char ip[64];
          inet_ntop(AF_INET, &ca.sin_addr, ip, sizeof(ip));
          c->addr = std::string(ip) + ":" + std::to_string(ntohs(ca.sin_port));
          epoll_event cev{};
          cev.events = EPOLLIN;
          cev.data.fd = cfd;
          epoll_ctl(g_epfd, EPOLL_CTL_ADD, cfd, &cev);
          g_clients[cfd] = std::move(c);
        }
        continue;
      }
      auto it = g_clients.find(fd);
      if (it == g_clients.end()) continue;
      Client& c = *it->second;
      if (events[e].events & (EPOLLIN | EPOLLHUP | EPOLLERR)) {
        while (true) {
          const ssize_t k = recv(fd, buf, sizeof(buf), 0);
          if (k > 0) { c.in.append(buf, (size_t)k); continue; }
          if (k == 0 || (errno != EAGAIN && errno != EWOULDBLOCK)) c.closing = true;
          break;
        }
        size_t pos = 0;
        while (true) {
          const int r = parse_one(c.in, pos, argvv);
          if (r == 0) break;
          if (r < 0) { w_err(c, "Protocol error"); c.closing = true; break; }
          cmd(c, argvv);
        }
        c.in.erase(0, pos);
      }
      // pub/sub may have queued output for other clients: flush everyone with data
      std::vector<int> to_close;
      for (auto& kv : g_clients) {
        if (!kv.second->out.empty()) flush_client(*kv.second);
        if (kv.second->closing && kv.second->out.empty()) to_close.push_back(kv.first);
      }
      for (int cfd : to_close) close_client(cfd);
    }
    if (g_cfg.save_interval_s > 0 && g_dirty &&
        Clock::now() - last_save > std::chrono::seconds(g_cfg.save_interval_s)) {
      save_snapshot();
      last_save = Clock::now();
    }
  }
  if (g_cfg.save_interval_s > 0 && g_dirty) save_snapshot();
  for (auto& kv : g_clients) close(kv.first);
  close(lfd);
  return 0;
}
