// Core definitions shared by every native translation unit of the MI355X MLlib engine.
//
// Replaces the reference's exit()-on-error model
// (mllib-dal/src/main/native/error_handling.cpp:30-57, which kills the executor JVM) with typed
// C++ exceptions that the Python bindings translate into Python exceptions.  No global mutable
// state lives here; everything per-fit hangs off a Context (runtime/context.h).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <sstream>
#include <stdexcept>
#include <string>

namespace oap {

// ---------------------------------------------------------------------------------------------
// Error hierarchy (mapped 1:1 onto oap_mllib_amd.errors.* in the bindings).
// ---------------------------------------------------------------------------------------------
class Error : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};
class DeviceError : public Error {  // HIP runtime / kernel failures
 public:
  using Error::Error;
};
class CommError : public Error {  // RCCL / host collective failures, watchdog timeouts
 public:
  using Error::Error;
};
class ConfigError : public Error {  // invalid arguments / shapes / configuration
 public:
  using Error::Error;
};
class OutOfMemoryError : public Error {  // arena budget exhausted
 public:
  using Error::Error;
};

namespace detail {
template <typename E>
[[noreturn]] inline void raise(const char* file, int line, const std::string& msg) {
  std::ostringstream os;
  os << msg << " [" << file << ":" << line << "]";
  throw E(os.str());
}
}  // namespace detail

#define OAP_HIP_CHECK(expr)                                                                    \
  do {                                                                                         \
    hipError_t _oap_e = (expr);                                                                \
    if (_oap_e != hipSuccess)                                                                  \
      ::oap::detail::raise<::oap::DeviceError>(__FILE__, __LINE__,                             \
                                               std::string(#expr) + " failed: " +              \
                                                   hipGetErrorString(_oap_e));                 \
  } while (0)

#define OAP_CHECK(cond, msg)                                                                   \
  do {                                                                                         \
    if (!(cond)) {                                                                             \
      std::ostringstream _oap_os;                                                              \
      _oap_os << msg;                                                                          \
      ::oap::detail::raise<::oap::ConfigError>(__FILE__, __LINE__, _oap_os.str());             \
    }                                                                                          \
  } while (0)

#define OAP_THROW(ExcType, msg)                                                                \
  do {                                                                                         \
    std::ostringstream _oap_os;                                                                \
    _oap_os << msg;                                                                            \
    ::oap::detail::raise<ExcType>(__FILE__, __LINE__, _oap_os.str());                          \
  } while (0)

// ---------------------------------------------------------------------------------------------
// Element types that cross the Python boundary and the collective layer.
// ---------------------------------------------------------------------------------------------
enum class DType : int { F32 = 0, F64 = 1, BF16 = 2, I32 = 3, I64 = 4, U8 = 5 };

inline size_t dtype_size(DType t) {
  switch (t) {
    case DType::F32: return 4;
    case DType::F64: return 8;
    case DType::BF16: return 2;
    case DType::I32: return 4;
    case DType::I64: return 8;
    case DType::U8: return 1;
  }
  return 0;
}

inline const char* dtype_name(DType t) {
  switch (t) {
    case DType::F32: return "f32";
    case DType::F64: return "f64";
    case DType::BF16: return "bf16";
    case DType::I32: return "i32";
    case DType::I64: return "i64";
    case DType::U8: return "u8";
  }
  return "?";
}

enum class ReduceOp : int { Sum = 0, Max = 1, Min = 2 };

// Where an algorithm runs.  CPU is the reference/fallback engine used when no MI355X is visible
// (and by the CPU test-suite); GPU is the HIP/MFMA engine.
enum class Backend : int { CPU = 0, GPU = 1 };

inline size_t round_up(size_t v, size_t m) { return (v + m - 1) / m * m; }
inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace oap
