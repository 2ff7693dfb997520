/*
 * CPU ORACLE (test infrastructure only) — deterministic inputs and hashing used by the
 * reference's tests: std::mt19937 / std::mt19937_64 (test_ntt.cu:192-199 seeds its inputs
 * with std::mt19937(0xdeadbeef + log_h + log_rate)) and MD5 over the u32 output stream
 * (test_ntt.cu:208-216). Both are restated from their public specifications
 * (Matsumoto-Nishimura MT19937 as in C++11 [rand.predef]; RFC 1321).
 */
#include <string.h>

#include "oracle.h"

/* ---- MT19937 (32-bit) ---- */
void orc_mt_seed(orc_mt19937* g, uint32_t seed) {
	g->mt[0] = seed;
	for (int i = 1; i < 624; i++) g->mt[i] = 1812433253u * (g->mt[i - 1] ^ (g->mt[i - 1] >> 30)) + (uint32_t)i;
	g->idx = 624;
}
uint32_t orc_mt_next(orc_mt19937* g) {
	if (g->idx >= 624) {
		for (int i = 0; i < 624; i++) {
			uint32_t y = (g->mt[i] & 0x80000000u) | (g->mt[(i + 1) % 624] & 0x7fffffffu);
			g->mt[i] = g->mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
		}
		g->idx = 0;
	}
	uint32_t y = g->mt[g->idx++];
	y ^= y >> 11;
	y ^= (y << 7) & 0x9d2c5680u;
	y ^= (y << 15) & 0xefc60000u;
	y ^= y >> 18;
	return y;
}

/* ---- MT19937-64 ---- */
void orc_mt64_seed(orc_mt19937_64* g, uint64_t seed) {
	g->mt[0] = seed;
	for (int i = 1; i < 312; i++)
		g->mt[i] = 6364136223846793005ull * (g->mt[i - 1] ^ (g->mt[i - 1] >> 62)) + (uint64_t)i;
	g->idx = 312;
}
uint64_t orc_mt64_next(orc_mt19937_64* g) {
	if (g->idx >= 312) {
		for (int i = 0; i < 312; i++) {
			uint64_t y = (g->mt[i] & 0xFFFFFFFF80000000ull) | (g->mt[(i + 1) % 312] & 0x7FFFFFFFull);
			g->mt[i] = g->mt[(i + 156) % 312] ^ (y >> 1) ^ ((y & 1ull) ? 0xB5026F5AA96619E9ull : 0ull);
		}
		g->idx = 0;
	}
	uint64_t y = g->mt[g->idx++];
	y ^= (y >> 29) & 0x5555555555555555ull;
	y ^= (y << 17) & 0x71D67FFFEDA60000ull;
	y ^= (y << 37) & 0xFFF7EEE000000000ull;
	y ^= y >> 43;
	return y;
}

void orc_mt_fill(uint32_t seed, uint32_t* out, size_t n) {
	orc_mt19937 g;
	orc_mt_seed(&g, seed);
	for (size_t i = 0; i < n; i++) out[i] = orc_mt_next(&g);
}

void orc_fill128(uint32_t seed0, uint64_t seed64_base, uint32_t* out, size_t n) {
	orc_mt19937 g;
	orc_mt_seed(&g, seed0);
	orc_mt19937_64 h[3];
	for (int j = 0; j < 3; j++) orc_mt64_seed(&h[j], seed64_base + (uint64_t)(j + 1));
	for (size_t i = 0; i < n; i++) {
		out[4 * i + 0] = orc_mt_next(&g);
		for (int j = 0; j < 3; j++) out[4 * i + 1 + j] = (uint32_t)orc_mt64_next(&h[j]);
	}
}

/* ---- MD5 (RFC 1321) ---- */
typedef struct {
	uint32_t s[4];
	uint64_t len;
	uint8_t buf[64];
	size_t fill;
} md5ctx;

static const uint32_t K[64] = {
	0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
	0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
	0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
	0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
	0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
	0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
	0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
	0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
static const int R[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 5, 9,  14, 20, 5, 9,
						  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
						  4, 11, 16, 23, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};

static inline uint32_t rotl(uint32_t x, int c) { return (x << c) | (x >> (32 - c)); }

static void md5_block(md5ctx* c, const uint8_t* p) {
	uint32_t m[16];
	for (int i = 0; i < 16; i++)
		m[i] = (uint32_t)p[4 * i] | ((uint32_t)p[4 * i + 1] << 8) | ((uint32_t)p[4 * i + 2] << 16) |
			   ((uint32_t)p[4 * i + 3] << 24);
	uint32_t a = c->s[0], b = c->s[1], cc = c->s[2], d = c->s[3];
	for (int i = 0; i < 64; i++) {
		uint32_t f;
		int g;
		if (i < 16) {
			f = (b & cc) | (~b & d);
			g = i;
		} else if (i < 32) {
			f = (d & b) | (~d & cc);
			g = (5 * i + 1) % 16;
		} else if (i < 48) {
			f = b ^ cc ^ d;
			g = (3 * i + 5) % 16;
		} else {
			f = cc ^ (b | ~d);
			g = (7 * i) % 16;
		}
		uint32_t t = d;
		d = cc;
		cc = b;
		b = b + rotl(a + f + K[i] + m[g], R[i]);
		a = t;
	}
	c->s[0] += a;
	c->s[1] += b;
	c->s[2] += cc;
	c->s[3] += d;
}
static void md5_init(md5ctx* c) {
	c->s[0] = 0x67452301;
	c->s[1] = 0xefcdab89;
	c->s[2] = 0x98badcfe;
	c->s[3] = 0x10325476;
	c->len = 0;
	c->fill = 0;
}
static void md5_update(md5ctx* c, const uint8_t* p, size_t n) {
	c->len += n;
	while (n) {
		size_t take = 64 - c->fill;
		if (take > n) take = n;
		memcpy(c->buf + c->fill, p, take);
		c->fill += take;
		p += take;
		n -= take;
		if (c->fill == 64) {
			md5_block(c, c->buf);
			c->fill = 0;
		}
	}
}
static void md5_final(md5ctx* c, uint8_t out[16]) {
	uint64_t bits = c->len * 8;
	uint8_t pad = 0x80;
	md5_update(c, &pad, 1);
	uint8_t z = 0;
	while (c->fill != 56) md5_update(c, &z, 1);
	uint8_t lb[8];
	for (int i = 0; i < 8; i++) lb[i] = (uint8_t)(bits >> (8 * i));
	md5_update(c, lb, 8);
	for (int i = 0; i < 4; i++)
		for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(c->s[i] >> (8 * j));
}

void orc_md5(const void* data, size_t len, uint8_t digest[16]) {
	md5ctx c;
	md5_init(&c);
	md5_update(&c, (const uint8_t*)data, len);
	md5_final(&c, digest);
}

void orc_md5_limb(const uint32_t* v, size_t n_elems, int limb, uint8_t digest[16]) {
	md5ctx c;
	md5_init(&c);
	uint32_t tmp[256];
	size_t i = 0;
	while (i < n_elems) {
		size_t k = 0;
		for (; k < 256 && i < n_elems; k++, i++) tmp[k] = v[4 * i + (size_t)limb];
		md5_update(&c, (const uint8_t*)tmp, 4 * k);
	}
	md5_final(&c, digest);
}
