// M31 / CM31 / QM31 (src/ulvt/finite_fields/m31.cuh:6-76, cm31.cuh:6-80, qm31.cuh:6-82), host
// mirror: M31 = GF(2^31 - 1), CM31 = M31[i]/(i^2 + 1), QM31 = CM31[u]/(u^2 - (2 + i)). Values are
// kept canonical (< 2^31 - 1; the reference may carry 2^31 - 1 for zero). A QM31 is 16 bytes in
// the reference's member order (lo.a, lo.b, hi.a, hi.b), which is the C-ABI's word order.
#pragma once

#include <cstdint>
#include <string>

class M31 {
public:
	static constexpr uint32_t BITS = 31;
	static constexpr uint32_t P = (1u << BITS) - 1;
	uint32_t val;

	constexpr M31() noexcept : val(0) {}
	constexpr M31(uint32_t v) noexcept : val(v % P) {}
	constexpr M31(uint64_t v) noexcept : val((uint32_t)(v % P)) {}  // m31.cuh:19-21 (any u64 here)

	constexpr M31 operator+(M31 r) const { return raw(val + r.val >= P ? val + r.val - P : val + r.val); }
	constexpr M31 operator-(M31 r) const { return raw(val >= r.val ? val - r.val : val + P - r.val); }
	constexpr M31 operator*(M31 r) const { return M31((uint64_t)val * r.val); }
	M31& operator+=(M31 r) { return *this = *this + r; }
	M31& operator-=(M31 r) { return *this = *this - r; }
	M31& operator*=(M31 r) { return *this = *this * r; }
	constexpr bool operator==(M31 r) const { return val == r.val; }
	constexpr bool operator!=(M31 r) const { return val != r.val; }
	std::string to_string() const { return std::to_string(val); }

private:
	static constexpr M31 raw(uint32_t v) {
		M31 m;
		m.val = v;
		return m;
	}
};

class CM31 {
public:
	M31 subfield_elements[2];

	constexpr CM31() noexcept : subfield_elements{M31(), M31()} {}
	constexpr CM31(uint32_t v) noexcept : subfield_elements{M31(v), M31()} {}
	constexpr CM31(const uint64_t v[2]) noexcept : subfield_elements{M31(v[0]), M31(v[1])} {}
	constexpr CM31(M31 lo, M31 hi) noexcept : subfield_elements{lo, hi} {}

	constexpr CM31 operator+(CM31 r) const {
		return CM31(subfield_elements[0] + r.subfield_elements[0], subfield_elements[1] + r.subfield_elements[1]);
	}
	constexpr CM31 operator-(CM31 r) const {
		return CM31(subfield_elements[0] - r.subfield_elements[0], subfield_elements[1] - r.subfield_elements[1]);
	}
	constexpr CM31 operator*(CM31 r) const {  // (a + bi)(c + di) = (ac - bd) + (ad + bc)i
		return CM31(subfield_elements[0] * r.subfield_elements[0] - subfield_elements[1] * r.subfield_elements[1],
					subfield_elements[0] * r.subfield_elements[1] + subfield_elements[1] * r.subfield_elements[0]);
	}
	CM31& operator+=(CM31 r) { return *this = *this + r; }
	CM31& operator-=(CM31 r) { return *this = *this - r; }
	CM31& operator*=(CM31 r) { return *this = *this * r; }
	constexpr bool operator==(CM31 r) const {
		return subfield_elements[0] == r.subfield_elements[0] && subfield_elements[1] == r.subfield_elements[1];
	}
	constexpr bool operator!=(CM31 r) const { return !(*this == r); }
	std::string to_string() const {
		return "(" + subfield_elements[0].to_string() + ", " + subfield_elements[1].to_string() + ")";
	}
};

class QM31 {
public:
	static constexpr uint32_t BITS = 31;
	static constexpr uint32_t P = (1u << BITS) - 1;
	CM31 subfield_elements[2];

	constexpr QM31() noexcept : subfield_elements{CM31(), CM31()} {}
	constexpr QM31(uint32_t v) noexcept : subfield_elements{CM31(v), CM31()} {}
	// QM31(uint64_t[4]) (qm31.cuh:22): exact component sums, reduced
	constexpr QM31(const uint64_t v[4]) noexcept : subfield_elements{CM31(v), CM31(v + 2)} {}
	constexpr QM31(CM31 lo, CM31 hi) noexcept : subfield_elements{lo, hi} {}

	constexpr QM31 operator+(QM31 r) const {
		return QM31(subfield_elements[0] + r.subfield_elements[0], subfield_elements[1] + r.subfield_elements[1]);
	}
	constexpr QM31 operator-(QM31 r) const {
		return QM31(subfield_elements[0] - r.subfield_elements[0], subfield_elements[1] - r.subfield_elements[1]);
	}
	// (lo + hi u)(lo' + hi' u) = lo lo' + R hi hi' + (lo hi' + hi lo') u, R = 2 + i (qm31.cuh:6, 38-43)
	constexpr QM31 operator*(QM31 r) const {
		return QM31(subfield_elements[0] * r.subfield_elements[0] + R() * subfield_elements[1] * r.subfield_elements[1],
					subfield_elements[0] * r.subfield_elements[1] + subfield_elements[1] * r.subfield_elements[0]);
	}
	QM31& operator+=(QM31 r) { return *this = *this + r; }
	QM31& operator-=(QM31 r) { return *this = *this - r; }
	QM31& operator*=(QM31 r) { return *this = *this * r; }
	constexpr bool operator==(QM31 r) const {
		return subfield_elements[0] == r.subfield_elements[0] && subfield_elements[1] == r.subfield_elements[1];
	}
	constexpr bool operator!=(QM31 r) const { return !(*this == r); }

	void write_to_u64(uint64_t dst[4]) const {
		for (int k = 0; k < 4; k++) dst[k] = subfield_elements[k / 2].subfield_elements[k % 2].val;
	}
	// C-ABI word order (lo.a, lo.b, hi.a, hi.b)
	void to_words(uint32_t w[4]) const {
		for (int k = 0; k < 4; k++) w[k] = subfield_elements[k / 2].subfield_elements[k % 2].val;
	}
	static QM31 from_words(const uint32_t w[4]) { return QM31(CM31(M31(w[0]), M31(w[1])), CM31(M31(w[2]), M31(w[3]))); }
	std::string to_string() const {
		return "(" + subfield_elements[0].to_string() + ", " + subfield_elements[1].to_string() + ")";
	}

private:
	static constexpr CM31 R() { return CM31(M31(2u), M31(1u)); }
};

static_assert(sizeof(QM31) == 16, "QM31 is four u32 words");
