#include "runtime/log.h"
#include "runtime/knobs.h"

#include <dlfcn.h>

#include <cstdio>
#include <cstdlib>
#include <sstream>

namespace oap {

namespace {
int64_t now_us() {
  return std::chrono::duration_cast<std::chrono::microseconds>(
             std::chrono::system_clock::now().time_since_epoch())
      .count();
}
const char* level_name(LogLevel l) {
  switch (l) {
    case LogLevel::Debug: return "debug";
    case LogLevel::Info: return "info";
    case LogLevel::Warn: return "warn";
    case LogLevel::Error: return "error";
    default: return "off";
  }
}
LogLevel level_from_env() {
  const std::string s = knob_str("OAP_MLLIB_LOG_LEVEL");
  if (s == "debug") return LogLevel::Debug;
  if (s == "info") return LogLevel::Info;
  if (s == "warn") return LogLevel::Warn;
  if (s == "error") return LogLevel::Error;
  if (s == "off") return LogLevel::Off;
  return LogLevel::Warn;
}
}  // namespace

Logger::Logger() {
  level_ = level_from_env();
  path_ = knob_str("OAP_MLLIB_LOG_FILE");
}

Logger& Logger::instance() {
  static Logger* inst = new Logger();  // intentionally leaked: usable during static teardown
  return *inst;
}

void Logger::configure(int rank, int device, LogLevel level, const std::string& path) {
  std::lock_guard<std::mutex> g(mu_);
  rank_ = rank;
  device_ = device;
  level_ = level;
  if (file_) {
    std::fclose(static_cast<FILE*>(file_));
    file_ = nullptr;
  }
  path_ = path;
}

void Logger::log(LogLevel lvl, const std::string& phase, const std::string& fields) {
  if (lvl < level_ || level_ == LogLevel::Off) return;
  std::ostringstream os;
  os << "{\"ts_us\":" << now_us() << ",\"rank\":" << rank_ << ",\"dev\":" << device_
     << ",\"level\":\"" << level_name(lvl) << "\",\"phase\":\"" << json_escape(phase) << "\"";
  if (!fields.empty()) os << "," << fields;
  os << "}\n";
  std::string line = os.str();
  std::lock_guard<std::mutex> g(mu_);
  FILE* out = stderr;
  if (!path_.empty()) {
    if (!file_) {
      std::string p = path_;
      auto pos = p.find("{rank}");
      if (pos != std::string::npos) p.replace(pos, 6, std::to_string(rank_));
      file_ = std::fopen(p.c_str(), "a");
    }
    if (file_) out = static_cast<FILE*>(file_);
  }
  std::fwrite(line.data(), 1, line.size(), out);
  std::fflush(out);
}

std::string json_escape(const std::string& s) {
  std::string o;
  o.reserve(s.size() + 2);
  for (char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\t': o += "\\t"; break;
      default:
        if (static_cast<unsigned char>(c) < 0x20) {
          char buf[8];
          std::snprintf(buf, sizeof(buf), "\\u%04x", c);
          o += buf;
        } else {
          o += c;
        }
    }
  }
  return o;
}

// ------------------------------------------------------------------------------------ Metrics
void Metrics::add(const std::string& phase, double us, int64_t bytes) {
  std::lock_guard<std::mutex> g(mu_);
  auto& s = phases_[phase];
  s.count += 1;
  s.total_us += us;
  if (us > s.max_us) s.max_us = us;
  s.bytes += bytes;
}
void Metrics::set_value(const std::string& name, double v) {
  std::lock_guard<std::mutex> g(mu_);
  values_[name] = v;
}
std::map<std::string, PhaseStat> Metrics::phases() const {
  std::lock_guard<std::mutex> g(mu_);
  return phases_;
}
std::map<std::string, double> Metrics::values() const {
  std::lock_guard<std::mutex> g(mu_);
  return values_;
}
void Metrics::reset() {
  std::lock_guard<std::mutex> g(mu_);
  phases_.clear();
  values_.clear();
}

// -------------------------------------------------------------------------------------- roctx
namespace {
struct Roctx {
  using push_fn = int (*)(const char*);
  using pop_fn = int (*)();
  using mark_fn = void (*)(const char*);
  push_fn push = nullptr;
  pop_fn pop = nullptr;
  mark_fn mark = nullptr;
  Roctx() {
    if (knob_on("OAP_MLLIB_NO_ROCTX")) return;
    const char* libs[] = {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                          "libroctx64.so.4", "libroctx64.so"};
    for (const char* l : libs) {
      void* h = dlopen(l, RTLD_NOW | RTLD_LOCAL | RTLD_NOLOAD);
      if (!h) h = dlopen(l, RTLD_NOW | RTLD_LOCAL);
      if (!h) continue;
      push = reinterpret_cast<push_fn>(dlsym(h, "roctxRangePushA"));
      pop = reinterpret_cast<pop_fn>(dlsym(h, "roctxRangePop"));
      mark = reinterpret_cast<mark_fn>(dlsym(h, "roctxMarkA"));
      if (push && pop) return;
      push = nullptr;
      pop = nullptr;
      mark = nullptr;
    }
  }
};
Roctx& roctx() {
  static Roctx r;
  return r;
}
}  // namespace

void roctx_push(const char* name) {
  if (auto f = roctx().push) f(name);
}
void roctx_pop() {
  if (auto f = roctx().pop) f();
}
void roctx_mark(const char* name) {
  if (auto f = roctx().mark) f(name);
}

// --------------------------------------------------------------------------------- TraceRange
TraceRange::TraceRange(Metrics* metrics, const char* phase, int64_t bytes, bool log)
    : metrics_(metrics), phase_(phase), bytes_(bytes), log_(log),
      t0_(std::chrono::steady_clock::now()) {
  roctx_push(phase);
}

double TraceRange::elapsed_us() const {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0_)
      .count();
}

TraceRange::~TraceRange() {
  roctx_pop();
  double us = elapsed_us();
  if (metrics_) metrics_->add(phase_, us, bytes_);
  if (log_) {
    std::ostringstream os;
    os << "\"us\":" << us << ",\"bytes\":" << bytes_;
    Logger::instance().log(LogLevel::Info, phase_, os.str());
  }
}

}  // namespace oap
