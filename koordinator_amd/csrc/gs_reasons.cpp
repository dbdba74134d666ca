// gs_reasons.cpp — the reference's Filter status (framework.Code + message) for a gs_evaluate failure code, so a
// cgo wrapper can return the same *framework.Status the plugins return.
//
//   NodeResourcesFit  [upstream] noderesources/fit.go fitsRequest: "Too many pods", "Insufficient cpu",
//                     "Insufficient memory", "Insufficient ephemeral-storage", "Insufficient <scalar>", joined by ", "
//                     (framework.Status.Message), Unschedulable
//   LoadAware         load_aware.go:45-46 ErrReasonUsageExceedThreshold / ErrReasonAggregatedUsageExceedThreshold
//                     with the resource (GS_FAIL_LA_MEMORY / GS_FAIL_LA_AGGREGATED), Unschedulable (:218-221, :250)
//   NodeNUMAResource  plugin.go:48-55 (Err* constants), util.go:117, topology_hint.go:36, topologymanager/manager.go:70,
//                     resource_manager.go:292,396 (the allocator's errors)
#include <stdio.h>
#include <string.h>

#include <string>

#include "../../include/gpuscore.h"

namespace {

constexpr int kSuccess = 0, kUnschedulable = 1, kUnresolvable = 2;

struct NumaReason {
  int code;
  const char* msg;
};
// indexed by gs_numa_reason
const NumaReason kNuma[] = {
    {kSuccess, ""},
    {kUnresolvable, "the requested CPUs must be integer"},                               // ErrInvalidRequestedCPUs
    {kUnresolvable, "node(s) invalid CPU amplification ratio"},                          // ErrInvalidCPUAmplificationRatio
    {kUnresolvable, "node(s) invalid CPU Topology"},                                     // GetAvailableCPUs error (:396)
    {kUnschedulable, "Insufficient amplified cpu"},                                      // ErrInsufficientAmplifiedCPU
    {kUnresolvable, "node(s) invalid CPU Topology"},                                     // ErrInvalidCPUTopology
    {kUnresolvable, "node(s) cpu bind policy conflicts with pod's required cpu bind policy"},   // ErrCPUBindPolicyConflict
    {kUnresolvable, "node(s) requested cpus not multiple cpus per core"},                // ErrSMTAlignmentError
    {kUnschedulable, "not enough cpus available to satisfy request"},                    // allocateCPUSet (:292)
    {kUnresolvable, "node(s) missing NUMA resources"},                                   // topology_hint.go:36
    {kUnschedulable, "node(s) NUMA Topology affinity error"},                            // manager.go:70
    {kUnschedulable, "not enough cpus available to satisfy request"},                    // Allocate after Admit (see gpuscore.h)
};

const char* const kScalarDefault[4] = {"kubernetes.io/batch-cpu", "kubernetes.io/batch-memory", "kubernetes.io/mid-cpu",
                                       "kubernetes.io/mid-memory"};

}  // namespace

extern "C" int gs_reason_string(uint32_t code, uint32_t scalar_mask, const char* const* scalar_names, char* buf,
                                size_t len) {
  const uint32_t known = GS_FAIL_FIT_PODS | GS_FAIL_FIT_CPU | GS_FAIL_FIT_MEMORY | GS_FAIL_FIT_EPHEMERAL |
                         GS_FAIL_FIT_SCALAR | GS_FAIL_LOADAWARE | GS_FAIL_NUMA_MASK | GS_FAIL_LA_MEMORY |
                         GS_FAIL_LA_AGGREGATED;
  const uint32_t numa = (code & GS_FAIL_NUMA_MASK) >> GS_FAIL_NUMA_SHIFT;
  if ((code & ~known) || numa >= sizeof(kNuma) / sizeof(kNuma[0])) return GS_EINVAL;
  if ((code & (GS_FAIL_LA_MEMORY | GS_FAIL_LA_AGGREGATED)) && !(code & GS_FAIL_LOADAWARE)) return GS_EINVAL;
  std::string msg;
  int status = kSuccess;
  const uint32_t fit = code & (GS_FAIL_FIT_PODS | GS_FAIL_FIT_CPU | GS_FAIL_FIT_MEMORY | GS_FAIL_FIT_EPHEMERAL |
                               GS_FAIL_FIT_SCALAR);
  if (fit) {   // the first plugin of the Filter order fails: its reasons, in fitsRequest order
    status = kUnschedulable;
    auto add = [&](const std::string& r) { msg += (msg.empty() ? "" : ", ") + r; };
    if (code & GS_FAIL_FIT_PODS) add("Too many pods");
    if (code & GS_FAIL_FIT_CPU) add("Insufficient cpu");
    if (code & GS_FAIL_FIT_MEMORY) add("Insufficient memory");
    if (code & GS_FAIL_FIT_EPHEMERAL) add("Insufficient ephemeral-storage");
    if (code & GS_FAIL_FIT_SCALAR)
      for (int s = 3; s < 7; ++s)
        if (scalar_mask >> s & 1u) add(std::string("Insufficient ") + (scalar_names ? scalar_names[s - 3] : kScalarDefault[s - 3]));
  } else if (code & GS_FAIL_LOADAWARE) {
    status = kUnschedulable;
    char tmp[96];
    snprintf(tmp, sizeof(tmp), (code & GS_FAIL_LA_AGGREGATED) ? "node(s) %s aggregated usage exceed threshold"
                                                              : "node(s) %s usage exceed threshold",
             (code & GS_FAIL_LA_MEMORY) ? "memory" : "cpu");
    msg = tmp;
  } else if (numa) {
    status = kNuma[numa].code;
    msg = kNuma[numa].msg;
  }
  if (buf && len) {
    const size_t n = msg.size() < len - 1 ? msg.size() : len - 1;
    memcpy(buf, msg.data(), n);
    buf[n] = '\0';
  }
  return status;
}
