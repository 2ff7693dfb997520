/*
 * CPU ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * QM31 (degree-4 extension of the Mersenne-31 field) sumcheck, restating the reference's
 * prime-field sibling: M31 / CM31 / QM31 arithmetic (src/ulvt/finite_fields/m31.cuh:6-76,
 * cm31.cuh:6-80, qm31.cuh:6-82: CM31 = M31[i]/(i^2+1), QM31 = CM31[u]/(u^2 - (2+i))), the round
 * messages of get_round_coefficients (src/ulvt/prime_field_sumcheck/core/kernels.cu:27-77:
 * points 0, 1, 2 of the product of the two columns' lines, summed per component as integers
 * and reduced, qm31.cuh:7 QM31(uint64_t[4])), fold_list_halves (kernels.cu:5-25:
 * lo <- lo + (hi - lo) * r) and interpolate_at (utils/interpolate.hpp:3-8). Values are kept
 * canonical (< 2^31 - 1); the reference may carry 2^31 - 1 for zero, which its sums and
 * products treat as zero, so the canonical results are the same.
 * There are no golden vectors for this path; it is pinned by the reference test's protocol
 * invariants (src/ulvt/prime_field_sumcheck/test_sumcheck.cu:9-99).
 */
#include "oracle.h"

#define M31_P 0x7fffffffu

static uint32_t m_add(uint32_t a, uint32_t b) {
	uint32_t s = a + b;
	return s >= M31_P ? s - M31_P : s;
}
static uint32_t m_sub(uint32_t a, uint32_t b) { return a >= b ? a - b : a + M31_P - b; }
static uint32_t m_mul(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) % M31_P); }

typedef struct { uint32_t a, b; } cm;          /* a + b i */
typedef struct { cm lo, hi; } qm;              /* lo + hi u */

static cm c_add(cm x, cm y) { return (cm){m_add(x.a, y.a), m_add(x.b, y.b)}; }
static cm c_sub(cm x, cm y) { return (cm){m_sub(x.a, y.a), m_sub(x.b, y.b)}; }
static cm c_mul(cm x, cm y) {
	return (cm){m_sub(m_mul(x.a, y.a), m_mul(x.b, y.b)), m_add(m_mul(x.a, y.b), m_mul(x.b, y.a))};
}
static qm q_add(qm x, qm y) { return (qm){c_add(x.lo, y.lo), c_add(x.hi, y.hi)}; }
static qm q_sub(qm x, qm y) { return (qm){c_sub(x.lo, y.lo), c_sub(x.hi, y.hi)}; }
static qm q_mul(qm x, qm y) {
	const cm R = {2, 1};
	return (qm){c_add(c_mul(x.lo, y.lo), c_mul(R, c_mul(x.hi, y.hi))), c_add(c_mul(x.lo, y.hi), c_mul(x.hi, y.lo))};
}
static qm q_load(const uint32_t* p) { return (qm){{p[0] % M31_P, p[1] % M31_P}, {p[2] % M31_P, p[3] % M31_P}}; }
static void q_store(uint32_t* p, qm v) {
	p[0] = v.lo.a;
	p[1] = v.lo.b;
	p[2] = v.hi.a;
	p[3] = v.hi.b;
}

void orc_qm31_mul(const uint32_t* a, const uint32_t* b, uint32_t* out) { q_store(out, q_mul(q_load(a), q_load(b))); }

/* one_half = QM31(0x40000000): challenge (challenge-1) e2 / 2 - challenge (challenge-2) e1
 * + (challenge-1)(challenge-2) e0 / 2 */
void orc_qm31_interpolate(const uint32_t* points /* 3 x 4 */, const uint32_t* r, uint32_t* out) {
	const qm c = q_load(r), one = {{1, 0}, {0, 0}}, two = {{2, 0}, {0, 0}}, half = {{0x40000000u, 0}, {0, 0}};
	const qm e0 = q_load(points), e1 = q_load(points + 4), e2 = q_load(points + 8);
	const qm cm1 = q_sub(c, one), cm2 = q_sub(c, two);
	qm t = q_mul(q_mul(q_mul(c, cm1), e2), half);
	t = q_sub(t, q_mul(q_mul(c, cm2), e1));
	t = q_add(t, q_mul(q_mul(q_mul(cm1, cm2), e0), half));
	q_store(out, t);
}

/* evals: 2 columns x 2^n QM31 (4 words each), modified in place. For each round i < n:
 * points[12 i .. 12 i + 11] = points 0, 1, 2 of the round, then fold with challenges[4 i ..]. */
void orc_qm31_sumcheck_run(uint32_t* evals, int n, const uint32_t* challenges, uint32_t* points) {
	const size_t N = (size_t)1 << n;
	uint32_t* col1 = evals + 4 * N;
	size_t cur = N;
	for (int i = 0; i < n; i++) {
		const size_t h = cur / 2;
		uint64_t s[3][4] = {{0}};
		for (size_t r = 0; r < h; r++) {
			const qm l0 = q_load(evals + 4 * r), u0 = q_load(evals + 4 * (r + h));
			const qm l1 = q_load(col1 + 4 * r), u1 = q_load(col1 + 4 * (r + h));
			const qm p[3] = {q_mul(l0, l1), q_mul(u0, u1),
			                 q_mul(q_add(q_sub(u0, l0), u0), q_add(q_sub(u1, l1), u1))};
			for (int k = 0; k < 3; k++) {
				s[k][0] += p[k].lo.a;
				s[k][1] += p[k].lo.b;
				s[k][2] += p[k].hi.a;
				s[k][3] += p[k].hi.b;
			}
		}
		for (int k = 0; k < 3; k++)
			for (int c = 0; c < 4; c++) points[12 * i + 4 * k + c] = (uint32_t)(s[k][c] % M31_P);
		const qm ch = q_load(challenges + 4 * i);
		for (size_t r = 0; r < h; r++) {
			uint32_t* cols[2] = {evals, col1};
			for (int j = 0; j < 2; j++) {
				const qm lo = q_load(cols[j] + 4 * r), hi = q_load(cols[j] + 4 * (r + h));
				q_store(cols[j] + 4 * r, q_add(lo, q_mul(q_sub(hi, lo), ch)));
			}
		}
		cur = h;
	}
}
