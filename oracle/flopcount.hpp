// flopcount.hpp - counts the algorithmic floating-point operations of the CPU oracle.
//
// TEST / MEASUREMENT INFRASTRUCTURE ONLY ("algorithmic FLOPs counted by
// instrumenting the CPU restatement"). oracle/flops.cpp includes this header, then
// pianosim_ref.c with `double` redefined to `fd`, a double that counts every arithmetic
// operation it takes part in. An operation with a zero operand is NOT counted (a*0, a+0,
// 0/a): the restatement keeps dense 140-wide rows and dense per-hand matrices for
// clarity, and skipping the zero operands turns its count into the sparse (structural)
// work of the algorithm, which is what the HIP kernel executes. Comparisons, fabs,
// floor/ceil and conversions are free; sqrt / divide / transcendental = 1 op each.
#pragma once
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <cmath>

extern "C" {
// [0] add/sub  [1] mul  [2] div  [3] sqrt + transcendentals + fmin/fmax
extern unsigned long long ref_flop_count[4];
}

struct fd {
  double v;
  fd() = default;
  constexpr fd(double x) : v(x) {}
  explicit operator double() const { return v; }
  explicit operator float() const { return (float)v; }
  explicit operator int() const { return (int)v; }
  explicit operator long() const { return (long)v; }
  explicit operator bool() const { return v != 0.0; }
};

inline void fc_count(int k, double a, double b) {
  if (a != 0.0 && b != 0.0) ref_flop_count[k]++;
}
inline void fc_count1(int k) { ref_flop_count[k]++; }

#define FC_BIN(OP, K)                                                                    \
  inline fd operator OP(fd a, fd b) { fc_count(K, a.v, b.v); return fd(a.v OP b.v); }     \
  inline fd operator OP(fd a, double b) { fc_count(K, a.v, b); return fd(a.v OP b); }     \
  inline fd operator OP(double a, fd b) { fc_count(K, a, b.v); return fd(a OP b.v); }     \
  inline fd& operator OP##=(fd& a, fd b) { fc_count(K, a.v, b.v); a.v = a.v OP b.v; return a; } \
  inline fd& operator OP##=(fd& a, double b) { fc_count(K, a.v, b); a.v = a.v OP b; return a; }
FC_BIN(+, 0)
FC_BIN(-, 0)
FC_BIN(*, 1)
FC_BIN(/, 2)
#undef FC_BIN
inline fd operator-(fd a) { return fd(-a.v); }
inline fd operator+(fd a) { return a; }

#define FC_CMP(OP)                                                      \
  inline bool operator OP(fd a, fd b) { return a.v OP b.v; }             \
  inline bool operator OP(fd a, double b) { return a.v OP b; }           \
  inline bool operator OP(double a, fd b) { return a OP b.v; }
FC_CMP(<)
FC_CMP(>)
FC_CMP(<=)
FC_CMP(>=)
FC_CMP(==)
FC_CMP(!=)
#undef FC_CMP

inline fd fabs(fd a) { return fd(::fabs(a.v)); }
inline fd floor(fd a) { return fd(::floor(a.v)); }
inline fd ceil(fd a) { return fd(::ceil(a.v)); }
inline fd round(fd a) { return fd(::round(a.v)); }
#define FC_UN(F) inline fd F(fd a) { fc_count1(3); return fd(::F(a.v)); }
FC_UN(sqrt)
FC_UN(exp)
FC_UN(log)
FC_UN(sin)
FC_UN(cos)
FC_UN(tan)
FC_UN(asin)
FC_UN(acos)
FC_UN(atan)
#undef FC_UN
#define FC_BI(F)                                                                     \
  inline fd F(fd a, fd b) { fc_count1(3); return fd(::F(a.v, b.v)); }                 \
  inline fd F(fd a, double b) { fc_count1(3); return fd(::F(a.v, b)); }               \
  inline fd F(double a, fd b) { fc_count1(3); return fd(::F(a, b.v)); }
FC_BI(fmax)
FC_BI(fmin)
FC_BI(pow)
FC_BI(atan2)
FC_BI(fmod)
FC_BI(hypot)
#undef FC_BI
inline fd copysign(fd a, fd b) { return fd(::copysign(a.v, b.v)); }
inline fd copysign(fd a, double b) { return fd(::copysign(a.v, b)); }
inline fd copysign(double a, fd b) { return fd(::copysign(a, b.v)); }

#define _Thread_local thread_local
#define double fd
