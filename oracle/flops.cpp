// flops.cpp - the CPU oracle compiled with a counting double (see flopcount.hpp).
// TEST / MEASUREMENT INFRASTRUCTURE ONLY: built into oracle/_build/liboracle_flops.so,
// loaded by tools/count_flops.py and tests/test_flops.py, never by the product.
#include "flopcount.hpp"

extern "C" {
unsigned long long ref_flop_count[4];
void ref_flops_reset(void) { memset(ref_flop_count, 0, sizeof(ref_flop_count)); }
void ref_flops_get(unsigned long long* out) { memcpy(out, ref_flop_count, sizeof(ref_flop_count)); }

#include "pianosim_ref.c"
}
