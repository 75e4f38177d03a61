// Floating-point operation counter for the CPU oracle (TEST / MEASUREMENT INFRASTRUCTURE ONLY).
//
// oracle/Makefile's `flops` target compiles ackphys_oracle.c as C++ with this header forced in
// first and `double` defined to `fd`: a double that counts its arithmetic per oracle stage
// (OR_STAGE markers in ackphys_oracle.c). The counts are the "algorithmic FLOPs per env-step" of
// what the reference's algorithm (MuJoCo's mj_step restated in f64, plus the env
// glue) executes, independent of how the GPU kernels restructure it. Counting rules: + - * / and
// sqrt are 1 FLOP each; the transcendental calls (sin, cos, tan, atan, atan2, exp, log, pow) are
// counted separately (1 each in `trans`); comparisons, fabs/fmin/fmax, copies and conversions are
// free. The layout is a plain double, so the C ABI (double* arrays, double returns) is unchanged.
#pragma once
// every system header the oracle includes, before `double` is redefined below
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>

namespace orf {
constexpr int NSTAGE = 16;
inline unsigned long long g_flops[NSTAGE];
inline unsigned long long g_trans[NSTAGE];
inline int g_stage = 0;
inline void add(unsigned long long n) { g_flops[g_stage] += n; }
inline void trans() { g_trans[g_stage] += 1; }
}  // namespace orf

struct fd {
  double v;
  fd() = default;
  template <class T, class = std::enable_if_t<std::is_arithmetic_v<T>>>
  constexpr fd(T x) : v((double)x) {}
  template <class T, class = std::enable_if_t<std::is_arithmetic_v<T>>>
  explicit constexpr operator T() const { return (T)v; }
  fd& operator+=(fd o) { orf::add(1); v += o.v; return *this; }
  fd& operator-=(fd o) { orf::add(1); v -= o.v; return *this; }
  fd& operator*=(fd o) { orf::add(1); v *= o.v; return *this; }
  fd& operator/=(fd o) { orf::add(1); v /= o.v; return *this; }
  fd operator-() const { return fd(-v); }
  fd operator+() const { return *this; }
  fd& operator++() { orf::add(1); v += 1; return *this; }
  fd& operator--() { orf::add(1); v -= 1; return *this; }
  fd operator++(int) { fd t = *this; orf::add(1); v += 1; return t; }
  fd operator--(int) { fd t = *this; orf::add(1); v -= 1; return t; }
};
static_assert(sizeof(fd) == sizeof(double) && std::is_trivially_copyable_v<fd>, "fd must be layout-compatible");

template <class T>
using fd_arg = std::enable_if_t<std::is_same_v<T, fd> || std::is_arithmetic_v<T>, fd>;
template <class A, class B>
constexpr bool fd_pair = (std::is_same_v<A, fd> || std::is_same_v<B, fd>) &&
                         (std::is_same_v<A, fd> || std::is_arithmetic_v<A>) &&
                         (std::is_same_v<B, fd> || std::is_arithmetic_v<B>);
inline double fdv(fd x) { return x.v; }
template <class T, class = std::enable_if_t<std::is_arithmetic_v<T>>>
inline double fdv(T x) { return (double)x; }

#define FD_BINOP(OP)                                          \
  template <class A, class B, class = std::enable_if_t<fd_pair<A, B>>> \
  inline fd operator OP(A a, B b) {                           \
    orf::add(1);                                              \
    return fd(fdv(a) OP fdv(b));                              \
  }
FD_BINOP(+)
FD_BINOP(-)
FD_BINOP(*)
FD_BINOP(/)
#undef FD_BINOP
#define FD_CMP(OP)                                            \
  template <class A, class B, class = std::enable_if_t<fd_pair<A, B>>> \
  inline bool operator OP(A a, B b) {                         \
    return fdv(a) OP fdv(b);                                  \
  }
FD_CMP(<)
FD_CMP(>)
FD_CMP(<=)
FD_CMP(>=)
FD_CMP(==)
FD_CMP(!=)
#undef FD_CMP
inline bool operator!(fd a) { return !a.v; }

// <math.h> on fd (free functions are not counted as FLOPs except sqrt; transcendentals apart)
inline fd sqrt(fd x) { orf::add(1); return fd(std::sqrt(x.v)); }
inline fd fabs(fd x) { return fd(std::fabs(x.v)); }
#define FD_TRANS1(F) \
  inline fd F(fd x) { orf::trans(); return fd(std::F(x.v)); }
FD_TRANS1(sin)
FD_TRANS1(cos)
FD_TRANS1(tan)
FD_TRANS1(atan)
FD_TRANS1(exp)
FD_TRANS1(log)
FD_TRANS1(asin)
FD_TRANS1(acos)
#undef FD_TRANS1
template <class A, class B, class = std::enable_if_t<fd_pair<A, B>>>
inline fd atan2(A y, B x) { orf::trans(); return fd(std::atan2(fdv(y), fdv(x))); }
template <class A, class B, class = std::enable_if_t<fd_pair<A, B>>>
inline fd pow(A x, B y) { orf::trans(); return fd(std::pow(fdv(x), fdv(y))); }
template <class A, class B, class = std::enable_if_t<fd_pair<A, B>>>
inline fd fmin(A a, B b) { return fd(std::fmin(fdv(a), fdv(b))); }
template <class A, class B, class = std::enable_if_t<fd_pair<A, B>>>
inline fd fmax(A a, B b) { return fd(std::fmax(fdv(a), fdv(b))); }
template <class A, class B, class = std::enable_if_t<fd_pair<A, B>>>
inline fd copysign(A a, B b) { return fd(std::copysign(fdv(a), fdv(b))); }
inline fd floor(fd x) { return fd(std::floor(x.v)); }
inline fd ceil(fd x) { return fd(std::ceil(x.v)); }
inline fd round(fd x) { return fd(std::round(x.v)); }
inline fd rint(fd x) { return fd(std::rint(x.v)); }
inline fd trunc(fd x) { return fd(std::trunc(x.v)); }
inline bool isnan(fd x) { return std::isnan(x.v); }
inline bool isinf(fd x) { return std::isinf(x.v); }
inline bool isfinite(fd x) { return std::isfinite(x.v); }

extern "C" {
// counters of the calling thread's stages (single-threaded use: nthreads = 1)
__attribute__((visibility("default"), used)) void or_flops_reset(void) {
  for (int i = 0; i < orf::NSTAGE; i++) orf::g_flops[i] = orf::g_trans[i] = 0;
}
__attribute__((visibility("default"), used)) int or_flops_read(unsigned long long* flops, unsigned long long* trans,
                                                              int n) {
  for (int i = 0; i < n && i < orf::NSTAGE; i++) {
    flops[i] = orf::g_flops[i];
    trans[i] = orf::g_trans[i];
  }
  return orf::NSTAGE;
}
}

#define OR_STAGE(k) (orf::g_stage = (k))
#define double fd
