/*
 * x86_sse_probe.c -- the host CPU's own SSE arithmetic, operand order fixed by
 * inline assembly, for pinning the oracle's NaN-payload rule (tests only).
 *
 * The reference's Op<float>/Op<double>::Sum/Prod and complex operator*=
 * (op.cpp:42-64, 289-300) run as scalar SSE instructions on x86-64.  The
 * oracle (oracle/msx_oracle.c X86_OP) restates their NaN behaviour as a rule;
 * these functions execute the instructions themselves, with the operand
 * written first in op.cpp as the instruction's first source (destination)
 * operand, so the compiler cannot commute them.  AT&T syntax: "addss y, x"
 * computes x = x + y.
 */
#include <stdint.h>

#define SSE_BIN(NAME, T, INSN)                                                 \
    static inline T NAME(T x, T y)                                             \
    {                                                                          \
        __asm__(INSN " %[y], %[x]" : [x] "+x"(x) : [y] "x"(y));                \
        return x;                                                              \
    }
SSE_BIN(add_f, float, "addss")
SSE_BIN(sub_f, float, "subss")
SSE_BIN(mul_f, float, "mulss")
SSE_BIN(add_d, double, "addsd")
SSE_BIN(sub_d, double, "subsd")
SSE_BIN(mul_d, double, "mulsd")
/* MAXSS x, y = (x > y) ? x : y and MINSS x, y = (x < y) ? x : y: the
 * Windows max/min macros op.cpp:26,38 apply to (inout, in) */
SSE_BIN(max_f, float, "maxss")
SSE_BIN(min_f, float, "minss")
SSE_BIN(max_d, double, "maxsd")
SSE_BIN(min_d, double, "minsd")

/* inout[i] = inout[i] op in[i] (op 0 = SUM, 1 = PROD, 2 = MAX, 3 = MIN) */
void sse_f32(int op, const float* in, float* inout, int64_t n)
{
    for (int64_t i = 0; i < n; ++i)
        inout[i] = op == 0 ? add_f(inout[i], in[i]) : op == 1 ? mul_f(inout[i], in[i])
                 : op == 2 ? max_f(inout[i], in[i]) : min_f(inout[i], in[i]);
}

void sse_f64(int op, const double* in, double* inout, int64_t n)
{
    for (int64_t i = 0; i < n; ++i)
        inout[i] = op == 0 ? add_d(inout[i], in[i]) : op == 1 ? mul_d(inout[i], in[i])
                 : op == 2 ? max_d(inout[i], in[i]) : min_d(inout[i], in[i]);
}

/* complex<T>::operator*= (op.cpp:294-303), pairs (re, im):
 *   re' = (re * rhs.re) - (im * rhs.im);  im' = (re * rhs.im) + (rhs.re * im) */
void sse_c32_prod(const float* in, float* inout, int64_t n)
{
    for (int64_t i = 0; i < n; ++i) {
        const float re = inout[2 * i], im = inout[2 * i + 1], rre = in[2 * i], rim = in[2 * i + 1];
        inout[2 * i] = sub_f(mul_f(re, rre), mul_f(im, rim));
        inout[2 * i + 1] = add_f(mul_f(re, rim), mul_f(rre, im));
    }
}

void sse_c64_prod(const double* in, double* inout, int64_t n)
{
    for (int64_t i = 0; i < n; ++i) {
        const double re = inout[2 * i], im = inout[2 * i + 1], rre = in[2 * i], rim = in[2 * i + 1];
        inout[2 * i] = sub_d(mul_d(re, rre), mul_d(im, rim));
        inout[2 * i + 1] = add_d(mul_d(re, rim), mul_d(rre, im));
    }
}
