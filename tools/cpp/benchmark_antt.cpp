// Additive-NTT harness in the format of the reference's benchmark_antt.cu (src/ulvt/ntt/tests/
// benchmark_antt.cu:143-238): GF(2^32), r = 0, log_h 1..MAX, reference-semantics apply()
// (host buffers in and out) timed for the two kernel variants, each checked against the
// reference MD5 table (passed in as `hashes.txt`: one "log_h hex" line per entry).
//   ./benchmark_antt hashes.txt [max_log_h]
// Column mapping: "Original" = variant 0 (compact tiles, twiddle recomputed per butterfly, as
// the reference kernel), "Modified" = variant 1 (bitsliced tiles, precomputed twiddle
// contributions; the reference's ModifiedAdditiveNTT idea without its indexing/leak bugs).
#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <sstream>
#include <iostream>
#include <map>
#include <random>
#include <string>

#include "ntt/additive_ntt.hpp"
#include "../../oracle/oracle.h"

using Clock = std::chrono::high_resolution_clock;

static std::string md5hex(const void* p, size_t n) {
	uint8_t d[16];
	orc_md5(p, n, d);
	char s[33];
	for (int i = 0; i < 16; i++) std::snprintf(s + 2 * i, 3, "%02x", d[i]);
	return s;
}

static std::string speedup(double r) {
	std::ostringstream o;
	o << std::fixed << std::setprecision(3) << r << "x";
	return o.str();
}

int main(int argc, char** argv) {
	if (argc < 2) {
		std::cerr << "usage: benchmark_antt hashes.txt [max_log_h]\n";
		return 2;
	}
	std::map<int, std::string> want;
	std::ifstream hf(argv[1]);
	int lh;
	std::string hx;
	while (hf >> lh >> hx) want[lh] = hx;
	const int max_log_h = argc > 2 ? std::atoi(argv[2]) : 28;
	std::cout << "\n====================================================================================\n"
			  << "                  ADDITIVE NTT BENCHMARK: Original vs Modified (r=0)\n"
			  << "====================================================================================\n"
			  << std::left << std::setw(8) << "log_h" << std::setw(15) << "Original (ms)" << std::setw(15)
			  << "Modified (ms)" << std::setw(12) << "Speedup" << std::setw(12) << "Orig.Valid" << std::setw(12)
			  << "Mod.Valid" << "\n"
			  << "------------------------------------------------------------------------------------\n";
	int pass[2] = {0, 0}, rows = 0;
	double total[2] = {0, 0};
	for (int log_h = 1; log_h <= max_log_h; log_h++) {
		std::mt19937 gen(0xdeadbeef + log_h);
		NTTData<uint32_t> in(DataOrder::IN_ORDER, (size_t)1 << log_h), out((size_t)1 << log_h);
		for (size_t i = 0; i < in.size; i++) in.data[i] = gen();
		AdditiveNTT<uint32_t, FanPaarTowerField<5>> ntt(AdditiveNTTConf<uint32_t, FanPaarTowerField<5>>(log_h, 0));
		double ms[2] = {-1, -1};
		bool ok[2] = {false, false};
		for (int v = 0; v < 2; v++) {
			if (v == 1 && log_h < 12) {  // the bitsliced tile needs 2^12 points: same kernel as v0
				ms[1] = ms[0];
				ok[1] = ok[0];
				break;
			}
			try {
				ntt.set_variant(v);
				ntt.apply(in, out);  // warm-up
				const auto t0 = Clock::now();
				const bool applied = ntt.apply(in, out);
				const auto t1 = Clock::now();
				ms[v] = std::chrono::duration<double, std::milli>(t1 - t0).count();
				ok[v] = applied && want.count(log_h) && md5hex(out.data.get(), out.byte_len()) == want[log_h];
			} catch (const std::exception& e) {
				std::cout << "log_h " << log_h << " variant " << v << ": " << e.what() << std::endl;
			}
		}
		rows++;
		for (int v = 0; v < 2; v++) pass[v] += ok[v], total[v] += ms[v];
		std::cout << std::left << std::setw(8) << log_h << std::fixed << std::setprecision(2) << std::setw(15) << ms[0]
				  << std::setw(15) << ms[1] << std::setw(12) << speedup(ms[0] / ms[1])
				  << std::setw(12) << (ok[0] ? "PASS" : "FAIL") << std::setw(12) << (ok[1] ? "PASS" : "FAIL") << std::endl;
	}
	std::cout << "====================================================================================\n"
			  << "SUMMARY:\n"
			  << "  Original tests passed: " << pass[0] << "/" << rows << "\n"
			  << "  Modified tests passed: " << pass[1] << "/" << rows << "\n"
			  << "  Total original time: " << std::fixed << std::setprecision(2) << total[0] << " ms\n"
			  << "  Total modified time: " << std::fixed << std::setprecision(2) << total[1] << " ms\n"
			  << "  Average speedup: " << std::fixed << std::setprecision(3) << total[0] / total[1] << "x\n";
	return (pass[0] == rows && pass[1] == rows) ? 0 : 1;
}
