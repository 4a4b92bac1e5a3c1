// AdjDbCodec.h — KvStore "adj:" values (compact-protocol AdjacencyDatabase) <-> the
// host mirror's thrift structs, in bulk.
//
// Reference path: Decision::processPublication
// (openr/decision/Decision.cpp:1737-1782) decodes every "adj:<node>" value with
// fbzmq::util::readThriftObjStr<thrift::AdjacencyDatabase>(value, serializer_), where
// serializer_ is apache::thrift::CompactSerializer (Decision.h:399), checks the node
// name against the key, stamps the area and calls LinkState::updateAdjacencyDatabase.
// LinkMonitor writes those values with writeThriftObjStr (LinkMonitor.cpp:620).
//
// The wire format is fbthrift's CompactProtocol (fbthrift rev f101a1f5, pinned at
// build/deps/github_hashes/facebook/fbthrift-rev.txt, not vendored): field headers
// with 4-bit id deltas (long form = type byte + zigzag-varint i16 id), zigzag varints
// for i16/i32/i64, varint-length binary, list headers with a 4-bit size (15 = varint
// size follows), booleans folded into the field-header type nibble. The schema is
// openr/if/Lsdb.thrift:24-32, :71-129 and Network.thrift:55-58.
//
// Here the decode is native C++ over std::string_view with no per-field allocation
// beyond the mirror structs, and many values decode in parallel on host threads; the
// mirror then builds the CSR for the GPU engine once per publication (the LinkState
// mirror is rebuilt lazily). Unknown fields of every compact type are skipped, as the
// generated fbthrift reader does.
//
// BinaryAddress.addr: the wire carries raw 4/16-byte addresses; the mirror keeps them
// as text (LinkState.h), so 4/16-byte values are converted with inet_ntop / inet_pton
// (an empty address stays empty, any other length is carried as raw bytes).
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

#include "LinkState.h"

namespace openr {

// TProtocolException-equivalent: malformed, truncated or over-deep input.
class CompactProtocolError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

namespace serializer {

// writeThriftObjStr(adjDb, CompactSerializer) — fields in IDL declaration order
// (Adjacency writes id 5 nextHopV4 before id 4 metric, exercising the long header).
std::string writeAdjacencyDatabase(const thrift::AdjacencyDatabase& db);

// readThriftObjStr<AdjacencyDatabase>(value, CompactSerializer). Trailing bytes after
// the struct's STOP are ignored, as Serializer::deserialize does.
thrift::AdjacencyDatabase readAdjacencyDatabase(std::string_view value);

// Bulk decode on `nThreads` host threads (0 = hardware concurrency). Output order =
// input order. Throws CompactProtocolError naming the first bad value's index.
std::vector<thrift::AdjacencyDatabase> readAdjacencyDatabases(const std::vector<std::string_view>& values,
                                                              unsigned nThreads = 0);

}  // namespace serializer

// The adjacency half of Decision::processPublication (Decision.cpp:1737-1782) for one
// area: keys starting with "adj:" are decoded (in bulk), checked against the node name
// in the key (CHECK_EQ there; std::invalid_argument here), stamped with `area` and
// applied with LinkState::updateAdjacencyDatabase in key order. Other keys are ignored
// (prefix:/fibtime: handling is outside the SPF path).
struct AdjPublicationResult {
  size_t adjDbsApplied = 0;
  bool topologyChanged = false;
  bool linkAttributesChanged = false;
  bool nodeLabelChanged = false;
};
AdjPublicationResult applyAdjacencyPublication(LinkState& linkState,
                                               const std::vector<std::pair<std::string, std::string>>& keyVals,
                                               unsigned nThreads = 0);

}  // namespace openr
