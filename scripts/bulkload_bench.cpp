// Host-only timing of the LinkState bulk load (decode -> updateAdjacencyDatabase per
// database -> CSR mirror), the linkstate_csr phase of `bench.py --workload adjdb`.
// Built and run by scripts/bulkload_prof.sh; no GPU needed (the engine is linked, not called).
#include <chrono>
#include <cstdio>
#include <fstream>
#include <iterator>

#include "AdjDbCodec.h"
#include "LinkState.h"

using namespace openr;
using Clock = std::chrono::steady_clock;

static double ms(Clock::time_point a, Clock::time_point b) {
  return std::chrono::duration<double, std::milli>(b - a).count();
}

int main(int argc, char** argv) {
  const char* dir = argc > 1 ? argv[1] : ".";
  const int iters = argc > 2 ? std::atoi(argv[2]) : 10;
  std::ifstream fd(std::string(dir) + "/data.bin", std::ios::binary), fo(std::string(dir) + "/off.bin", std::ios::binary);
  const std::string data((std::istreambuf_iterator<char>(fd)), {});
  const std::string o((std::istreambuf_iterator<char>(fo)), {});
  if (o.size() < 16) {
    std::fprintf(stderr, "no input in %s\n", dir);
    return 1;
  }
  const uint64_t* off = reinterpret_cast<const uint64_t*>(o.data());
  const size_t n = o.size() / 8 - 1;
  std::vector<std::string_view> vals;
  for (size_t i = 0; i < n; ++i) vals.emplace_back(data.data() + off[i], off[i + 1] - off[i]);
  double best[3] = {1e30, 1e30, 1e30};
  size_t E = 0;
  for (int it = 0; it < iters; ++it) {
    const auto t0 = Clock::now();
    auto dbs = serializer::readAdjacencyDatabases(vals, 1);
    const auto t1 = Clock::now();
    LinkState ls("0");
    for (auto& db : dbs) {
      db.area = "0";
      ls.updateAdjacencyDatabase(std::move(db), 0, 0);
    }
    const auto t2 = Clock::now();
    E = ls.csrMirror().col.size();
    const auto t3 = Clock::now();
    best[0] = std::min(best[0], ms(t0, t1));
    best[1] = std::min(best[1], ms(t1, t2));
    best[2] = std::min(best[2], ms(t2, t3));
  }
  std::printf("dbs %zu dir_edges %zu best of %d: decode(1 thr) %.1f ms update %.1f ms mirror %.1f ms\n", n, E, iters,
              best[0], best[1], best[2]);
  return 0;
}
