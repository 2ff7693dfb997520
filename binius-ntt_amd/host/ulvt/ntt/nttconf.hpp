// NTTData / DataOrder / AdditiveNTTConf (src/ulvt/ntt/nttconf.cuh:9-21, 49-114), host mirror.
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <stdexcept>

enum class DataOrder : char { INVALID = -1, IN_ORDER, BIT_REVERSED };

template <typename E>
class NTTData {
public:
	DataOrder order;
	std::unique_ptr<E[]> data;
	size_t size;

	NTTData(DataOrder order, size_t size) : order(order), data(std::make_unique<E[]>(size)), size(size) {}
	NTTData(size_t size) : order(DataOrder::INVALID), data(std::make_unique<E[]>(size)), size(size) {}
	inline size_t byte_len() const { return sizeof(E) * size; }
};

// The reference ASSERTs these (nttconf.cuh:55-60: abort in Debug); the mirror throws.
template <typename T, typename P>
class AdditiveNTTConf {
public:
	int log_h;
	int log_rate;

	AdditiveNTTConf(int log_h, int log_rate) : log_h(log_h), log_rate(log_rate) {
		if (!(log_h >= 1)) throw std::invalid_argument("AdditiveNTTConf: log_h >= 1");
		if (!(log_h + log_rate <= (int)P::N_BITS())) throw std::invalid_argument("AdditiveNTTConf: log_h + log_rate <= N_BITS");
		if (!(log_rate >= 0 && log_rate <= 4)) throw std::invalid_argument("AdditiveNTTConf: 0 <= log_rate <= 4");
	}
};
