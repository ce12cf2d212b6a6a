#include "runtime/knobs.h"

#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>

#include "runtime/common.h"

namespace oap {

namespace {
// (name, default, meaning) — the complete list of what the native layer reads
const std::vector<KnobInfo> kKnobs = {
    // ---- K-Means
    {"OAP_KMEANS_PROVISIONAL_MIN", "268435456",
     "elements (global rows x d) from which the fixed-point scales come from the initial centers "
     "(checked by the first pass) instead of a column-maxima pass up front"},
    {"OAP_KMEANS_ABSMAX_PASS", "0", "1: always take the column-maxima pass up front"},
    {"OAP_KMEANS_ROW_SCAN", "1",
     "0: the tile-level Hamerly scan instead of the image kernel's fused row scan"},
    {"OAP_KMEANS_IMAGE", "1", "0: no resident fp16 operand image (every pass reads f32 rows)"},
    {"OAP_KMEANS_REFINE", "1", "0: the worst-case tier-1 deferral test (no per-row residuals)"},
    {"OAP_KMEANS_EXACT", "",
     "exact re-decision of deferred rows: '' by size, 'mfma' the f32 MFMA sweep, 'cand' by "
     "candidates"},
    {"OAP_KMEANS_FINAL_COST", "",
     "'rows': the final cost of a costless last pass by a pass over the rows, not the statistics"},
    {"OAP_KMEANS_NO_LEAN_CHUNKED", "0",
     "1: large k (beyond one LDS plan) takes the general chunked kernel, not the lean one"},
    {"OAP_KMEANS_NO_WIDE", "0", "1: d > 128 takes the generic kernel, not the wide MFMA one"},
    {"OAP_KMEANS_INIT_PRECISE", "0", "1: k-means|| passes on the general (bf16x3) kernel"},
    {"OAP_KMEANS_INIT_SUPER", "",
     "k-means|| super-chunks of > 1 LDS plan of candidates: '' on, 0 off, 1 cost updates only, "
     "2 candidate counts only"},
    {"OAP_KMEANS_CHUNK_DEFER", "",
     "chunked passes: 0 re-decides in-chunk near ties at once instead of deferring them"},
    {"OAP_KMEANS_HOST_MARKS", "0", "1: host timestamps of a fit's phases to stderr"},
    // ---- ALS
    {"OAP_ALS_LD", "0", "factor row stride (floats; a multiple of 16 >= rank, <= 128; 0: rank"
                        " rounded up to 16)"},
    {"OAP_ALS_HOST_SETUP", "0", "1: ratings re-indexing and CSR build on the host"},
    {"OAP_ALS_LOWRANK", "1", "0: every short implicit row on the direct r x r solve"},
    {"OAP_ALS_GRAM", "", "'fp32': long-row Gramian chunks on exact-fp32 MFMA, not split fp16"},
    {"OAP_ALS_X3_MIN_LEN", "128", "direct rows longer than this use the split-fp16 Gramian"},
    {"OAP_ALS_DIRECT_X3", "1", "0: direct rows keep the exact-fp32 Gramian"},
    {"OAP_ALS_ABLATE", "0", "timing ablations of the ALS solve kernels (bit mask)"},
    {"OAP_ALS_LR3_OCC", "0", "waves per SIMD of the 33-48-rating low-rank class (0: default)"},
    {"OAP_ALS_ROTATE_VALU", "0", "1: factor rotations on the VALU instead of MFMA"},
    // ---- PCA
    {"OAP_PCA_EXACT_ENGINE", "int8",
     "exact mode on f32 rows: 'int8' digit products on the int8 MFMA (error bound reported), "
     "'fp64' fp64 products on the fp64 MFMA"},
    {"OAP_PCA_DIGIT_CHUNK_BYTES", "17179869184",
     "int8 exact engine: digit planes of one row chunk at most this many bytes (and a third of "
     "the free HBM)"},
    {"OAP_EIG_GRID", "0", "workgroups of the fused tridiagonalisation (0: one per CU)"},
    {"OAP_EIG_HOST_INVIT", "0", "1: inverse iteration on the host thread pool"},
    // ---- collectives, fault injection, logging
    {"OAP_RCCL_A2A_CHUNK_BYTES", "268435456", "RCCL alltoallv round size (bytes)"},
    {"OAP_TCP_PIECE_BYTES", "67108864", "TCP host-comm forwarding piece (bytes)"},
    {"OAP_MLLIB_FAULT", "", "fault injection 'rank:phase:iteration'"},
    {"OAP_MLLIB_FAULT_MODE", "raise", "'raise' a CommError or 'exit' the process"},
    {"OAP_MLLIB_LOG_LEVEL", "warn", "debug | info | warn | error | off"},
    {"OAP_MLLIB_LOG_FILE", "", "JSON-lines log file ('{rank}' substituted; '' stderr)"},
    {"OAP_MLLIB_NO_ROCTX", "0", "1: no roctx ranges"},
};

std::mutex g_mu;
std::map<std::string, std::string>& overrides() {
  static auto* m = new std::map<std::string, std::string>();  // (usable during teardown)
  return *m;
}

const KnobInfo& info(const char* name) {
  for (const KnobInfo& k : kKnobs)
    if (std::strcmp(k.name, name) == 0) return k;
  OAP_THROW(ConfigError, "unknown native knob " << name << " (runtime/knobs.cpp)");
}
}  // namespace

const std::vector<KnobInfo>& knob_table() { return kKnobs; }

std::string knob_str(const char* name) {
  const KnobInfo& k = info(name);
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = overrides().find(name);
    if (it != overrides().end()) return it->second;
  }
  const char* e = std::getenv(name);  // the one place the native layer reads the environment
  return e && *e ? std::string(e) : std::string(k.def);
}

int64_t knob_int(const char* name) {
  const std::string v = knob_str(name);
  char* end = nullptr;
  const long long x = std::strtoll(v.c_str(), &end, 10);
  if (v.empty() || end == v.c_str()) return std::strtoll(info(name).def, nullptr, 10);
  return x;
}

double knob_float(const char* name) {
  const std::string v = knob_str(name);
  char* end = nullptr;
  const double x = std::strtod(v.c_str(), &end);
  if (v.empty() || end == v.c_str()) return std::strtod(info(name).def, nullptr);
  return x;
}

bool knob_on(const char* name) {
  const std::string v = knob_str(name);
  return !v.empty() && v != "0";
}

void set_knob(const std::string& name, const std::string& value) {
  (void)info(name.c_str());
  std::lock_guard<std::mutex> g(g_mu);
  if (value.empty())
    overrides().erase(name);
  else
    overrides()[name] = value;
}

void clear_knobs() {
  std::lock_guard<std::mutex> g(g_mu);
  overrides().clear();
}

}  // namespace oap
