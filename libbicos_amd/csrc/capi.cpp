// capi.cpp -- the reference's ctypes C-ABI (src/pybicos_c.cpp:27-211), served by
// the gfx950 engine. Host buffers in, malloc'd host copies out.
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/bicos/common.hpp"
#include "../../include/bicos/match.hpp"
#include "../../include/bicos_c.h"
#include "engine.hpp"

namespace {

// reference src/pybicos_c.cpp:56-89 (convertConfig)
BICOS::Config convert_config(const BicosConfig* c) {
    BICOS::Config config;
    if (c->nxcorr_threshold >= 0) config.nxcorr_threshold = c->nxcorr_threshold;
    if (c->subpixel_step >= 0) config.subpixel_step = c->subpixel_step;
    if (c->min_variance >= 0) config.min_variance = c->min_variance;
    config.mode = c->mode == 0 ? BICOS::TransformMode::LIMITED : BICOS::TransformMode::FULL;
    config.precision = c->precision == 0 ? BICOS::Precision::SINGLE : BICOS::Precision::DOUBLE;
    if (c->variant_type == 0) {
        config.variant = BICOS::Variant::NoDuplicates{};
    } else {
        BICOS::Variant::Consistency consistency;
        consistency.max_lr_diff = c->max_lr_diff;
        consistency.no_dupes = c->no_dupes != 0;
        config.variant = consistency;
    }
    return config;
}

void* copy_out(const BICOS::Image& m) {
    const size_t bytes = (size_t)m.rows() * m.cols() * m.elemSize();
    void* p = std::malloc(bytes ? bytes : 1);
    if (!p) throw BICOS::Exception("out of host memory");
    for (int r = 0; r < m.rows(); ++r)
        std::memcpy((char*)p + (size_t)r * m.cols() * m.elemSize(), m.ptr<char>(r),
                    (size_t)m.cols() * m.elemSize());
    return p;
}

}  // namespace

extern "C" {

// reference src/pybicos_c.cpp:92-108
BicosConfig* BICOS_CreateDefaultConfig(void) {
    BicosConfig* config = (BicosConfig*)std::calloc(1, sizeof(BicosConfig));
    if (!config) return nullptr;
    config->nxcorr_threshold = 0.5f;
    config->subpixel_step = -1.0f;
    config->min_variance = -1.0f;
    config->mode = 0;
    config->precision = 0;
    config->variant_type = 0;
    config->max_lr_diff = 1;
    config->no_dupes = 0;
    return config;
}

void BICOS_FreeConfig(BicosConfig* config) { std::free(config); }

// Frees the result AND its buffers (the reference leaked the buffers).
void BICOS_FreeResult(BicosResult* result) {
    if (!result) return;
    std::free(result->disparity_data);
    std::free(result->corrmap_data);
    std::free(result);
}

// reference src/pybicos_c.cpp:131-200
BicosResult* BICOS_Match(void** stack0_data, int* stack0_rows, int* stack0_cols, int* stack0_types,
                         int stack0_size, void** stack1_data, int* stack1_rows, int* stack1_cols,
                         int* stack1_types, int stack1_size, BicosConfig* config) {
    BicosResult* result = nullptr;
    try {
        if (!config) throw BICOS::Exception("null config");
        if (stack0_size < 0 || stack1_size < 0) throw BICOS::Exception("negative stack size");
        std::vector<BICOS::Image> s0, s1;
        for (int i = 0; i < stack0_size; ++i)
            s0.emplace_back(stack0_rows[i], stack0_cols[i], stack0_types[i], stack0_data[i]);
        for (int i = 0; i < stack1_size; ++i)
            s1.emplace_back(stack1_rows[i], stack1_cols[i], stack1_types[i], stack1_data[i]);

        const BICOS::Config cc = convert_config(config);
        result = (BicosResult*)std::calloc(1, sizeof(BicosResult));
        if (!result) throw BICOS::Exception("out of host memory");
        // The result buffers are malloc'd as in the reference (pybicos_c.cpp:176,192) and
        // handed to BICOS::match as views, which it fills in place (Image::create keeps a
        // buffer of the right size and type), so nothing is copied after the download.
        BICOS::Image disparity, corrmap;
        if (stack0_size > 0 && stack0_rows[0] > 0 && stack0_cols[0] > 0) {
            const int rows = stack0_rows[0], cols = stack0_cols[0];
            const int dtype = cc.nxcorr_threshold ? BICOS::F32 : BICOS::S16;
            const int ctype = cc.precision == BICOS::Precision::DOUBLE ? BICOS::F64 : BICOS::F32;
            const size_t px = (size_t)rows * cols;
            result->disparity_data = std::malloc(px * BICOS::Image::elem_size(dtype));
            result->corrmap_data = std::malloc(px * BICOS::Image::elem_size(ctype));
            if (!result->disparity_data || !result->corrmap_data)
                throw BICOS::Exception("out of host memory");
            disparity = BICOS::Image(rows, cols, dtype, result->disparity_data);
            corrmap = BICOS::Image(rows, cols, ctype, result->corrmap_data);
        }
        BICOS::match(s0, s1, disparity, cc, &corrmap);

        // (only if match chose different buffers, e.g. empty images)
        if (disparity.data() != result->disparity_data) {
            std::free(result->disparity_data);
            result->disparity_data = nullptr;
            result->disparity_data = copy_out(disparity);
        }
        if (corrmap.data() != result->corrmap_data) {
            std::free(result->corrmap_data);
            result->corrmap_data = nullptr;
            result->corrmap_data = copy_out(corrmap);
        }
        result->disparity_rows = disparity.rows();
        result->disparity_cols = disparity.cols();
        result->disparity_type = disparity.type();
        result->corrmap_rows = corrmap.rows();
        result->corrmap_cols = corrmap.cols();
        result->corrmap_type = corrmap.type();
        return result;
    } catch (const std::exception& e) {
        bicos_impl::set_error(BICOS_E_ARG, e.what());
    } catch (...) {
        bicos_impl::set_error(BICOS_E_INTERNAL, "unknown exception");
    }
    BICOS_FreeResult(result);
    return nullptr;
}

// reference src/pybicos_c.cpp:203-209
float BICOS_InvalidDisparityFloat(void) { return BICOS::INVALID_DISP<float>; }
int16_t BICOS_InvalidDisparityInt16(void) { return BICOS::INVALID_DISP<int16_t>; }

}  // extern "C"
