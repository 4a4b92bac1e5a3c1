// AdjDbCodec.cpp — compact-protocol AdjacencyDatabase codec and the bulk adjacency
// publication path (see AdjDbCodec.h for the reference call sites).
#include "AdjDbCodec.h"

#include <arpa/inet.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>

namespace openr {
namespace {

// fbthrift CompactProtocol type nibbles (detail::compact::Types)
enum CType : uint8_t {
  CT_STOP = 0,
  CT_BOOL_TRUE = 1,
  CT_BOOL_FALSE = 2,
  CT_BYTE = 3,
  CT_I16 = 4,
  CT_I32 = 5,
  CT_I64 = 6,
  CT_DOUBLE = 7,
  CT_BINARY = 8,
  CT_LIST = 9,
  CT_SET = 10,
  CT_MAP = 11,
  CT_STRUCT = 12,
  CT_FLOAT = 13,
};
constexpr int kMaxDepth = 64;  // nesting bound for skip() on hostile input

// --------------------------------------------------------------------------- writer
class Writer {
 public:
  std::string out;

  void varint(uint64_t v) {
    while (v >= 0x80) {
      out.push_back(char(uint8_t(v) | 0x80));
      v >>= 7;
    }
    out.push_back(char(uint8_t(v)));
  }
  void i32(int32_t v) { varint(uint32_t((uint32_t(v) << 1) ^ uint32_t(v >> 31))); }
  void i64(int64_t v) { varint((uint64_t(v) << 1) ^ uint64_t(v >> 63)); }
  void binary(std::string_view s) {
    varint(s.size());
    out.append(s.data(), s.size());
  }
  void fieldHeader(uint8_t type, int16_t id) {
    const int delta = int(id) - int(last_);
    if (delta > 0 && delta <= 15) {
      out.push_back(char(uint8_t(delta << 4) | type));
    } else {
      out.push_back(char(type));
      varint(uint32_t((uint32_t(int32_t(id)) << 1) ^ uint32_t(int32_t(id) >> 31)));
    }
    last_ = id;
  }
  void boolField(int16_t id, bool v) { fieldHeader(v ? CT_BOOL_TRUE : CT_BOOL_FALSE, id); }
  void listHeader(uint8_t elemType, size_t n) {
    if (n < 15) {
      out.push_back(char(uint8_t(n << 4) | elemType));
    } else {
      out.push_back(char(0xf0 | elemType));
      varint(n);
    }
  }
  int16_t beginStruct() {
    const int16_t saved = last_;
    last_ = 0;
    return saved;
  }
  void endStruct(int16_t saved) {
    out.push_back(char(CT_STOP));
    last_ = saved;
  }

 private:
  int16_t last_ = 0;
};

std::string addrToWire(const std::string& text) {
  if (text.empty()) return {};
  unsigned char buf[16];
  if (text.find(':') != std::string::npos && inet_pton(AF_INET6, text.c_str(), buf) == 1) {
    return std::string(reinterpret_cast<char*>(buf), 16);
  }
  if (inet_pton(AF_INET, text.c_str(), buf) == 1) return std::string(reinterpret_cast<char*>(buf), 4);
  return text;  // not an address: carried as raw bytes (see header)
}

std::string addrFromWire(std::string_view raw) {
  char buf[INET6_ADDRSTRLEN];
  if (raw.size() == 16 && inet_ntop(AF_INET6, raw.data(), buf, sizeof(buf))) return buf;
  if (raw.size() == 4 && inet_ntop(AF_INET, raw.data(), buf, sizeof(buf))) return buf;
  return std::string(raw);
}

// Network.thrift:55-58
void writeBinaryAddress(Writer& w, const thrift::BinaryAddress& a) {
  const int16_t s = w.beginStruct();
  w.fieldHeader(CT_BINARY, 1);
  w.binary(addrToWire(a.addr));
  if (a.ifName) {
    w.fieldHeader(CT_BINARY, 3);
    w.binary(*a.ifName);
  }
  w.endStruct(s);
}

// Lsdb.thrift:71-110, IDL declaration order
void writeAdjacency(Writer& w, const thrift::Adjacency& a) {
  const int16_t s = w.beginStruct();
  w.fieldHeader(CT_BINARY, 1);
  w.binary(a.otherNodeName);
  w.fieldHeader(CT_BINARY, 2);
  w.binary(a.ifName);
  w.fieldHeader(CT_STRUCT, 3);
  writeBinaryAddress(w, a.nextHopV6);
  w.fieldHeader(CT_STRUCT, 5);
  writeBinaryAddress(w, a.nextHopV4);
  w.fieldHeader(CT_I32, 4);
  w.i32(a.metric);
  w.fieldHeader(CT_I32, 6);
  w.i32(a.adjLabel);
  w.boolField(7, a.isOverloaded);
  w.fieldHeader(CT_I32, 8);
  w.i32(a.rtt);
  w.fieldHeader(CT_I64, 9);
  w.i64(a.timestamp);
  w.fieldHeader(CT_I64, 10);
  w.i64(a.weight);
  w.fieldHeader(CT_BINARY, 11);
  w.binary(a.otherIfName);
  w.endStruct(s);
}

// Lsdb.thrift:24-32
void writePerfEvents(Writer& w, const thrift::PerfEvents& p) {
  const int16_t s = w.beginStruct();
  w.fieldHeader(CT_LIST, 1);
  w.listHeader(CT_STRUCT, p.events.size());
  for (const auto& e : p.events) {
    const int16_t se = w.beginStruct();
    w.fieldHeader(CT_BINARY, 1);
    w.binary(e.nodeName);
    w.fieldHeader(CT_BINARY, 2);
    w.binary(e.eventDescr);
    w.fieldHeader(CT_I64, 3);
    w.i64(e.unixTs);
    w.endStruct(se);
  }
  w.endStruct(s);
}

// --------------------------------------------------------------------------- reader
class Reader {
 public:
  explicit Reader(std::string_view in) : p_(reinterpret_cast<const uint8_t*>(in.data())), end_(p_ + in.size()) {}

  [[noreturn]] static void fail(const char* what) { throw CompactProtocolError(what); }

  uint8_t byte() {
    if (p_ == end_) fail("truncated input");
    return *p_++;
  }
  uint64_t varint(int maxBytes) {
    uint64_t v = 0;
    for (int shift = 0, i = 0; i < maxBytes; ++i, shift += 7) {
      const uint8_t b = byte();
      v |= uint64_t(b & 0x7f) << shift;
      if (!(b & 0x80)) return v;
    }
    fail("varint too long");
  }
  int16_t i16() {
    const uint32_t u = uint32_t(varint(3));
    return int16_t(int32_t(u >> 1) ^ -int32_t(u & 1));
  }
  int32_t i32() {
    const uint32_t u = uint32_t(varint(5));
    return int32_t(u >> 1) ^ -int32_t(u & 1);
  }
  int64_t i64() {
    const uint64_t u = varint(10);
    return int64_t(u >> 1) ^ -int64_t(u & 1);
  }
  std::string_view binary() {
    const uint64_t n = varint(5);
    if (n > uint64_t(end_ - p_)) fail("binary length exceeds input");
    std::string_view s(reinterpret_cast<const char*>(p_), size_t(n));
    p_ += n;
    return s;
  }
  void skipBytes(size_t n) {
    if (n > size_t(end_ - p_)) fail("truncated input");
    p_ += n;
  }

  // Returns false at STOP. `type` is the raw nibble (bool fields carry their value).
  bool fieldHeader(int16_t& last, uint8_t& type, int16_t& id) {
    const uint8_t b = byte();
    type = b & 0x0f;
    if (type == CT_STOP) return false;
    const uint8_t delta = b >> 4;
    id = delta ? int16_t(last + delta) : i16();
    last = id;
    return true;
  }
  // list/set header: element count and element type
  uint32_t listHeader(uint8_t& elemType) {
    const uint8_t b = byte();
    elemType = b & 0x0f;
    uint64_t n = b >> 4;
    if (n == 15) n = varint(5);
    // every element occupies at least one byte (bool / byte / varint / header)
    if (n > uint64_t(end_ - p_)) fail("container size exceeds input");
    return uint32_t(n);
  }

  // skip one value of compact type `type`; `inField` folds booleans into the header
  void skip(uint8_t type, bool inField, int depth) {
    if (depth > kMaxDepth) fail("nesting too deep");
    switch (type) {
      case CT_BOOL_TRUE:
      case CT_BOOL_FALSE:
        if (!inField) byte();
        return;
      case CT_BYTE:
        byte();
        return;
      case CT_I16:
      case CT_I32:
      case CT_I64:
        varint(10);
        return;
      case CT_DOUBLE:
        skipBytes(8);
        return;
      case CT_FLOAT:
        skipBytes(4);
        return;
      case CT_BINARY:
        binary();
        return;
      case CT_LIST:
      case CT_SET: {
        uint8_t et;
        const uint32_t n = listHeader(et);
        for (uint32_t i = 0; i < n; ++i) skip(et, false, depth + 1);
        return;
      }
      case CT_MAP: {
        const uint64_t n = varint(5);
        if (n == 0) return;
        if (n > uint64_t(end_ - p_)) fail("container size exceeds input");
        const uint8_t kv = byte();
        for (uint64_t i = 0; i < n; ++i) {
          skip(kv >> 4, false, depth + 1);
          skip(kv & 0x0f, false, depth + 1);
        }
        return;
      }
      case CT_STRUCT: {
        int16_t last = 0, id;
        uint8_t t;
        while (fieldHeader(last, t, id)) skip(t, true, depth + 1);
        return;
      }
      default:
        fail("unknown compact type");
    }
  }

 private:
  const uint8_t* p_;
  const uint8_t* end_;
};

inline bool isBoolType(uint8_t t) { return t == CT_BOOL_TRUE || t == CT_BOOL_FALSE; }

void readBinaryAddress(Reader& r, thrift::BinaryAddress& a, int depth) {
  int16_t last = 0, id;
  uint8_t t;
  bool haveAddr = false;
  while (r.fieldHeader(last, t, id)) {
    if (id == 1 && t == CT_BINARY) {
      a.addr = addrFromWire(r.binary());
      haveAddr = true;
    } else if (id == 3 && t == CT_BINARY) {
      a.ifName = std::string(r.binary());
    } else {
      r.skip(t, true, depth + 1);
    }
  }
  // `1: required binary addr` — the generated reader rejects a missing required field
  if (!haveAddr) Reader::fail("required field 'addr' of BinaryAddress missing");
}

void readAdjacency(Reader& r, thrift::Adjacency& a, int depth) {
  int16_t last = 0, id;
  uint8_t t;
  while (r.fieldHeader(last, t, id)) {
    switch (id) {
      case 1:
        if (t == CT_BINARY) { a.otherNodeName = std::string(r.binary()); continue; }
        break;
      case 2:
        if (t == CT_BINARY) { a.ifName = std::string(r.binary()); continue; }
        break;
      case 3:
        if (t == CT_STRUCT) { readBinaryAddress(r, a.nextHopV6, depth + 1); continue; }
        break;
      case 5:
        if (t == CT_STRUCT) { readBinaryAddress(r, a.nextHopV4, depth + 1); continue; }
        break;
      case 4:
        if (t == CT_I32) { a.metric = r.i32(); continue; }
        break;
      case 6:
        if (t == CT_I32) { a.adjLabel = r.i32(); continue; }
        break;
      case 7:
        if (isBoolType(t)) { a.isOverloaded = t == CT_BOOL_TRUE; continue; }
        break;
      case 8:
        if (t == CT_I32) { a.rtt = r.i32(); continue; }
        break;
      case 9:
        if (t == CT_I64) { a.timestamp = r.i64(); continue; }
        break;
      case 10:
        if (t == CT_I64) { a.weight = r.i64(); continue; }
        break;
      case 11:
        if (t == CT_BINARY) { a.otherIfName = std::string(r.binary()); continue; }
        break;
      default:
        break;
    }
    r.skip(t, true, depth + 1);  // unknown id or mismatched type
  }
}

void readPerfEvents(Reader& r, thrift::PerfEvents& p, int depth) {
  int16_t last = 0, id;
  uint8_t t;
  while (r.fieldHeader(last, t, id)) {
    if (id == 1 && t == CT_LIST) {
      uint8_t et;
      const uint32_t n = r.listHeader(et);
      if (et != CT_STRUCT) {
        for (uint32_t i = 0; i < n; ++i) r.skip(et, false, depth + 1);
        continue;
      }
      p.events.clear();
      p.events.resize(n);
      for (auto& e : p.events) {
        int16_t l2 = 0, id2;
        uint8_t t2;
        while (r.fieldHeader(l2, t2, id2)) {
          if (id2 == 1 && t2 == CT_BINARY) e.nodeName = std::string(r.binary());
          else if (id2 == 2 && t2 == CT_BINARY) e.eventDescr = std::string(r.binary());
          else if (id2 == 3 && t2 == CT_I64) e.unixTs = r.i64();
          else r.skip(t2, true, depth + 2);
        }
      }
    } else {
      r.skip(t, true, depth + 1);
    }
  }
}

void readAdjacencyDatabaseImpl(Reader& r, thrift::AdjacencyDatabase& db) {
  int16_t last = 0, id;
  uint8_t t;
  while (r.fieldHeader(last, t, id)) {
    switch (id) {
      case 1:
        if (t == CT_BINARY) { db.thisNodeName = std::string(r.binary()); continue; }
        break;
      case 2:
        if (isBoolType(t)) { db.isOverloaded = t == CT_BOOL_TRUE; continue; }
        break;
      case 3:
        if (t == CT_LIST) {
          uint8_t et;
          const uint32_t n = r.listHeader(et);
          if (et != CT_STRUCT) {
            for (uint32_t i = 0; i < n; ++i) r.skip(et, false, 1);
            continue;
          }
          db.adjacencies.clear();
          db.adjacencies.resize(n);
          for (auto& a : db.adjacencies) readAdjacency(r, a, 1);
          continue;
        }
        break;
      case 4:
        if (t == CT_I32) { db.nodeLabel = r.i32(); continue; }
        break;
      case 5:
        if (t == CT_STRUCT) {
          db.perfEvents.emplace();
          readPerfEvents(r, *db.perfEvents, 1);
          continue;
        }
        break;
      case 6:
        if (t == CT_BINARY) { db.area = std::string(r.binary()); continue; }
        break;
      default:
        break;
    }
    r.skip(t, true, 1);
  }
}

// Util.cpp:1042-1049 getNodeNameFromKey: folly::split(":") and take element 1
std::string nodeNameFromKey(const std::string& key) {
  const size_t a = key.find(':');
  if (a == std::string::npos) return "";
  const size_t b = key.find(':', a + 1);
  return key.substr(a + 1, b == std::string::npos ? std::string::npos : b - a - 1);
}

}  // namespace

namespace serializer {

std::string writeAdjacencyDatabase(const thrift::AdjacencyDatabase& db) {
  Writer w;
  w.out.reserve(64 + db.adjacencies.size() * 96);
  const int16_t s = w.beginStruct();
  w.fieldHeader(CT_BINARY, 1);
  w.binary(db.thisNodeName);
  w.boolField(2, db.isOverloaded);
  w.fieldHeader(CT_LIST, 3);
  w.listHeader(CT_STRUCT, db.adjacencies.size());
  for (const auto& a : db.adjacencies) writeAdjacency(w, a);
  w.fieldHeader(CT_I32, 4);
  w.i32(db.nodeLabel);
  if (db.perfEvents) {
    w.fieldHeader(CT_STRUCT, 5);
    writePerfEvents(w, *db.perfEvents);
  }
  w.fieldHeader(CT_BINARY, 6);
  w.binary(db.area);
  w.endStruct(s);
  return std::move(w.out);
}

thrift::AdjacencyDatabase readAdjacencyDatabase(std::string_view value) {
  thrift::AdjacencyDatabase db;
  Reader r(value);
  readAdjacencyDatabaseImpl(r, db);
  return db;
}

std::vector<thrift::AdjacencyDatabase> readAdjacencyDatabases(const std::vector<std::string_view>& values,
                                                              unsigned nThreads) {
  std::vector<thrift::AdjacencyDatabase> out(values.size());
  if (nThreads == 0) nThreads = std::max(1u, std::thread::hardware_concurrency());
  nThreads = unsigned(std::min<size_t>(nThreads, std::max<size_t>(1, values.size() / 64)));
  std::atomic<size_t> next{0};
  std::atomic<size_t> firstBad{values.size()};
  std::string badWhat;
  std::atomic_flag badLock = ATOMIC_FLAG_INIT;
  auto work = [&] {
    constexpr size_t kChunk = 32;
    for (;;) {
      const size_t lo = next.fetch_add(kChunk);
      if (lo >= values.size()) return;
      const size_t hi = std::min(values.size(), lo + kChunk);
      for (size_t i = lo; i < hi; ++i) {
        try {
          Reader r(values[i]);
          readAdjacencyDatabaseImpl(r, out[i]);
        } catch (const CompactProtocolError& e) {
          while (badLock.test_and_set()) {
          }
          if (i < firstBad.load()) {
            firstBad.store(i);
            badWhat = e.what();
          }
          badLock.clear();
        }
      }
    }
  };
  if (nThreads <= 1) {
    work();
  } else {
    std::vector<std::thread> pool;
    pool.reserve(nThreads - 1);
    for (unsigned t = 1; t < nThreads; ++t) pool.emplace_back(work);
    work();
    for (auto& th : pool) th.join();
  }
  if (firstBad.load() < values.size()) {
    throw CompactProtocolError("value " + std::to_string(firstBad.load()) + ": " + badWhat);
  }
  return out;
}

}  // namespace serializer

AdjPublicationResult applyAdjacencyPublication(LinkState& linkState,
                                               const std::vector<std::pair<std::string, std::string>>& keyVals,
                                               unsigned nThreads) {
  static const std::string kAdjDbMarker = "adj:";  // Constants.h:201
  std::vector<size_t> idx;
  std::vector<std::string_view> values;
  for (size_t i = 0; i < keyVals.size(); ++i) {
    if (keyVals[i].first.compare(0, kAdjDbMarker.size(), kAdjDbMarker) == 0) {
      idx.push_back(i);
      values.emplace_back(keyVals[i].second);
    }
  }
  auto dbs = serializer::readAdjacencyDatabases(values, nThreads);
  AdjPublicationResult res;
  for (size_t j = 0; j < dbs.size(); ++j) {
    const std::string nodeName = nodeNameFromKey(keyVals[idx[j]].first);
    if (nodeName != dbs[j].thisNodeName) {  // CHECK_EQ at Decision.cpp:1759
      throw std::invalid_argument("adj key " + keyVals[idx[j]].first + " carries node " + dbs[j].thisNodeName);
    }
    dbs[j].area = linkState.getArea();  // Decision.cpp:1762
    const auto change = linkState.updateAdjacencyDatabase(std::move(dbs[j]), 0, 0);
    res.topologyChanged |= change.topologyChanged;
    res.linkAttributesChanged |= change.linkAttributesChanged;
    res.nodeLabelChanged |= change.nodeLabelChanged;
    ++res.adjDbsApplied;
  }
  return res;
}

}  // namespace openr
