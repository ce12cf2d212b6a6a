// Structured per-rank logging, metrics and roctx tracing.
//
// The reference logs with std::cout at 1-second granularity
// (mllib-dal/src/main/native/KMeansDALImpl.cpp:202,218-222) and prints whole numeric tables
// (PCADALImpl.cpp:162-167).  Here every record is one JSON line
//   {"ts_us":..,"rank":..,"dev":..,"level":"info","phase":"kmeans/iter","us":..,"bytes":..,...}
// written to stderr or $OAP_MLLIB_LOG_FILE (with "{rank}" substituted), and every timed phase is
// also a roctx range so it shows up in `rocprofv3 --marker-trace` next to the kernels.
#pragma once

#include <chrono>
#include <cstdint>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace oap {

enum class LogLevel : int { Debug = 0, Info = 1, Warn = 2, Error = 3, Off = 4 };

class Logger {
 public:
  static Logger& instance();
  void configure(int rank, int device, LogLevel level, const std::string& path);
  LogLevel level() const { return level_; }
  int rank() const { return rank_; }
  // `fields` is a pre-rendered JSON fragment (without braces), e.g. "\"k\":200,\"d\":50".
  void log(LogLevel lvl, const std::string& phase, const std::string& fields);

 private:
  Logger();
  std::mutex mu_;
  int rank_ = 0;
  int device_ = -1;
  LogLevel level_ = LogLevel::Warn;
  std::string path_;
  void* file_ = nullptr;  // FILE*
};

// Escapes a string for embedding in a JSON document.
std::string json_escape(const std::string& s);

// Accumulating per-context metrics (phase -> {count, total_us, bytes}).
struct PhaseStat {
  int64_t count = 0;
  double total_us = 0.0;
  double max_us = 0.0;
  int64_t bytes = 0;
};

class Metrics {
 public:
  void add(const std::string& phase, double us, int64_t bytes = 0);
  void set_value(const std::string& name, double v);
  std::map<std::string, PhaseStat> phases() const;
  std::map<std::string, double> values() const;
  void reset();

 private:
  mutable std::mutex mu_;
  std::map<std::string, PhaseStat> phases_;
  std::map<std::string, double> values_;
};

// roctx markers, resolved lazily with dlopen so the library has no link-time dependency on a
// tracer (rocprofv3 provides librocprofiler-sdk-roctx; torch ships the legacy libroctx64).
void roctx_push(const char* name);
void roctx_pop();
void roctx_mark(const char* name);

// RAII range: roctx push/pop + host wall-clock into Metrics (+ optional log line).
class TraceRange {
 public:
  TraceRange(Metrics* metrics, const char* phase, int64_t bytes = 0, bool log = false);
  ~TraceRange();
  double elapsed_us() const;

 private:
  Metrics* metrics_;
  const char* phase_;
  int64_t bytes_;
  bool log_;
  std::chrono::steady_clock::time_point t0_;
};

}  // namespace oap
