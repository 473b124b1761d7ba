// Internal declarations shared by the translation units of liblbic.so.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "lbic.h"

namespace lbic {

int set_error(int code, const std::string& msg);

// GaussianConditional buffers after update() (entropy_layers_cai.py:590-613).
struct EntropyTables {
    int n_tables = 0;
    int stride = 0;                 // row stride of `cdf`
    std::vector<float> table;       // scale table (64)
    std::vector<int32_t> cdf;       // [n_tables][stride]
    std::vector<int32_t> length;    // cdf_length
    std::vector<int32_t> offset;    // -pmf_center
};

int pmf_to_quantized_cdf(const float* pmf, int n, int precision, uint32_t* cdf);
int rans_encode(const EntropyTables& t, const int32_t* symbols, const int32_t* indexes, size_t n,
                std::vector<uint8_t>& out);
int rans_decode_host(const EntropyTables& t, const uint8_t* data, size_t len, const int32_t* indexes, size_t n,
                     int32_t* out);

int build_rans_gpu_tables(const EntropyTables& t, std::vector<uint16_t>& img, std::vector<int>& meta);

}  // namespace lbic
