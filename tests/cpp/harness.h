// harness.h — the tiny test harness shared by the C++ host tests (no gtest in this
// image): EXPECT_* macros, TEST_CPU / TEST_GPU registration, and a main that runs the
// "cpu" or "gpu" group (or "all") and prints "N tests, M checks, F failures".
#pragma once

#include <cstdio>
#include <exception>
#include <functional>
#include <string>
#include <vector>

inline int g_failures = 0, g_checks = 0;
#define EXPECT_TRUE(c)                                                   \
  do {                                                                   \
    ++g_checks;                                                          \
    if (!(c)) {                                                          \
      ++g_failures;                                                      \
      std::fprintf(stderr, "  FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
    }                                                                    \
  } while (0)
#define EXPECT_FALSE(c) EXPECT_TRUE(!(c))
#define EXPECT_EQ(a, b) EXPECT_TRUE((a) == (b))
#define EXPECT_THROW(stmt)  \
  do {                      \
    bool thrown = false;    \
    try {                   \
      stmt;                 \
    } catch (...) {         \
      thrown = true;        \
    }                       \
    EXPECT_TRUE(thrown);    \
  } while (0)

struct TestCase {
  const char* name;
  bool gpu;
  std::function<void()> fn;
};
inline std::vector<TestCase>& registry() {
  static std::vector<TestCase> r;
  return r;
}
struct Reg {
  Reg(const char* n, bool gpu, std::function<void()> f) { registry().push_back({n, gpu, std::move(f)}); }
};
#define TEST_CPU(name) \
  static void name();  \
  static Reg reg_##name(#name, false, name);  \
  static void name()
#define TEST_GPU(name) \
  static void name();  \
  static Reg reg_##name(#name, true, name);  \
  static void name()


#ifndef OPENR_TEST_BUILD_ID
#define OPENR_TEST_BUILD_ID "unknown"
#endif

// extern "C" so the test binaries can read the libraries' build ids without the headers
extern "C" const char* openr_spf_build_id(void);
extern "C" const char* openr_decision_build_id(void);

inline int run_tests(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "cpu";
  // provenance (Makefile build_id): this binary's sources and the libraries it loaded
  std::printf("build-id: %s\n", OPENR_TEST_BUILD_ID);
  std::printf("engine-build-id: %s\n", openr_spf_build_id());
  std::printf("host-build-id: %s\n", openr_decision_build_id());
  if (mode == "build-id") return 0;
  int ran = 0;
  for (auto const& t : registry()) {
    if (t.gpu != (mode == "gpu") && mode != "all") continue;
    const int before = g_failures;
    try {
      t.fn();
    } catch (const std::exception& e) {
      ++g_failures;
      std::fprintf(stderr, "  EXCEPTION in %s: %s\n", t.name, e.what());
    }
    std::printf("[%s] %s\n", g_failures == before ? "PASS" : "FAIL", t.name);
    ++ran;
  }
  std::printf("%d tests, %d checks, %d failures\n", ran, g_checks, g_failures);
  return g_failures ? 1 : 0;
}
