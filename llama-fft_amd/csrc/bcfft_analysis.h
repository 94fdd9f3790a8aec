// bcfft_analysis.h — measurement scaffolding of the analysis builds, in one place.
//
// Product builds (make, libbcfft.so) define none of BCFFT_ABLATE / BCFFT_STAMPS / BCFFT_MARKS, and
// every macro below expands to nothing: the kernels' code objects are the same with or without
// these call sites (tools/isa_snapshot.sh compares them). The analysis builds are
//   make stamps  -DBCFFT_STAMPS   per-wave s_memtime phase stamps, product control flow
//                                 (tools/timeline_*.py read them through bcfft_set_stamps_*)
//   make ablate  -DBCFFT_ABLATE   stamps + phase switches set by bcfft_set_ablation*() (results
//                                 are WRONG when a switch is set: timing only)
//   -DBCFFT_MARKS                 ";MARK" comments in the ISA at the sub-phase points
//                                 (tools/isa_phases.py)
// Memory-only / compute-only builds of bc_forward_dm_kernel (-DBCFFT_DM_MEMONLY / -DBCFFT_DM_NOMEM)
// and the per-kernel ablation bits (-DBCFFT_*_ABL) are the same kind of build: they drop work and
// give wrong results by design.
#pragma once

#if defined(BCFFT_ABLATE) || defined(BCFFT_STAMPS)
#define BCFFT_ANALYSIS 1
// phase switches and the stamp buffer (static: each translation unit has its own copy and its
// own setter). ANALYSIS_INIT reads both ONCE per kernel into scalars: a per-use read would be a
// global load + s_waitcnt vmcnt(0) that drains every in-flight store and DMA, i.e. the measurement
// would serialise the kernel.
namespace bcfft {
static __device__ int g_ablate;
static __device__ unsigned long long* g_stamps;
}  // namespace bcfft
#define ANALYSIS_INIT                                                                          \
  const int ablate_flags_ = __builtin_amdgcn_readfirstlane(bcfft::g_ablate);                   \
  unsigned long long* const stamps_ = bcfft::g_stamps;                                         \
  (void)ablate_flags_;                                                                         \
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory")
#ifdef BCFFT_ABLATE
#define ABLATE(bit) (ablate_flags_ & (bit))
#else                                  // stamps-only build: the product's control flow, timed
#define ABLATE(bit) 0
#endif
#define STAMP_SLOTS 64
#define STAMP(id)                                                                              \
  do {                                                                                         \
    if (stamps_ && (threadIdx.x & 63) == 0) {                                                  \
      unsigned long long t_;                                                                   \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_) :: "memory");           \
      stamps_[((size_t)(blockIdx.y * gridDim.x + blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6)) \
          * STAMP_SLOTS + (id)] = t_;                                                          \
    }                                                                                          \
  } while (0)
// the stamp-buffer setter of one translation unit: extern "C" int bcfft_set_stamps_<name>(void*)
#define BCFFT_STAMPS_SETTER(name)                                                              \
  extern "C" int bcfft_set_stamps_##name(void* buf) {                                          \
    unsigned long long* p = (unsigned long long*)buf;                                          \
    return hipMemcpyToSymbol(HIP_SYMBOL(bcfft::g_stamps), &p, sizeof(p)) == hipSuccess ? 0 : BCFFT_ERR_HIP; \
  }
#else
#define ANALYSIS_INIT do {} while (0)
#define ABLATE(bit) 0
#define STAMP(id) do {} while (0)
#define BCFFT_STAMPS_SETTER(name)
#endif

// sub-phase stamps of one chosen iteration (the kernel keeps a bool `sub_on`), and ISA marks
#ifdef BCFFT_MARKS
#define SUBSTAMP(id) do { asm volatile(";MARK s" #id); if (sub_on) STAMP(id); } while (0)
#define MARK(id) asm volatile(";MARK " #id)
#else
#define SUBSTAMP(id) do { if (sub_on) STAMP(id); } while (0)
#define MARK(id) do {} while (0)
#endif
