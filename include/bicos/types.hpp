// bicos/types.hpp -- public types of the MI355X BICOS engine.
//
// Mirrors the reference's include/common.hpp (Config :73-82, Variant :63-71,
// INVALID_DISP :34-37, is_invalid :39-48, Exception :84-90) without OpenCV:
// `BICOS::HipImage` stands where cv::Mat / cv::cuda::GpuMat stand in the reference
// (:50-56) -- a small single-channel 2-D image that lives in host OR device (HBM) memory.
// Which type is spelled `BICOS::Image` is decided by the header a caller includes:
//   <bicos/common.hpp>  (native API)          Image = HipImage
//   <BICOS/common.hpp>  (the reference's installed header, include/BICOS/)
//                       Image = cv::Mat when <opencv2/core.hpp> exists (the reference's CPU
//                       build), else HipImage
#pragma once

#include <cmath>
#include <cstddef>
#include <cstdint>
#include <exception>
#include <limits>
#include <memory>
#include <optional>
#include <string>
#include <type_traits>
#include <variant>

// hipStream_t exactly as <hip/hip_runtime_api.h> declares it (an identical typedef may be
// repeated), so the API headers need no ROCm include path.
struct ihipStream_t;
typedef struct ihipStream_t* hipStream_t;

namespace BICOS {

// reference include/common.hpp:32
using uint128_t = __uint128_t;

template <typename T>
constexpr T INVALID_DISP = std::numeric_limits<T>::has_quiet_NaN
                               ? std::numeric_limits<T>::quiet_NaN()
                               : std::numeric_limits<T>::lowest();

template <typename T>
constexpr bool is_invalid(T disparity) {
    if constexpr (std::is_floating_point_v<T>)
        return std::isnan(disparity);
    else
        return disparity == INVALID_DISP<T>;
}

enum class TransformMode { LIMITED, FULL };
enum class Precision { SINGLE, DOUBLE };

namespace Variant {
struct NoDuplicates {};
struct Consistency {
    int max_lr_diff = 1;
    bool no_dupes = false;
};
}  // namespace Variant

using SearchVariant = std::variant<Variant::NoDuplicates, Variant::Consistency>;

// The reference's CUDA-build layout (common.hpp:73-82): `precision` sits between `mode` and
// `variant` and is always declared here (the library is compiled with it, and Config crosses
// the API by value). A caller written for the reference's CPU build that aggregate-initialises
// Config POSITIONALLY past `mode` must name the fields instead (`cfg.variant = ...`, or C++20
// designated initialisers `{.nxcorr_threshold = 0.9f, .variant = ...}`): the CPU build has no
// `precision`, so its fifth positional element is the variant. INTEGRATION.md s3.
struct Config {
    std::optional<float> nxcorr_threshold = 0.5f;
    std::optional<float> subpixel_step = std::nullopt;
    std::optional<float> min_variance = std::nullopt;
    TransformMode mode = TransformMode::LIMITED;
    Precision precision = Precision::SINGLE;
    SearchVariant variant = Variant::NoDuplicates{};
};

class Exception : public std::exception {
    std::string _message;

public:
    explicit Exception(const std::string& message) : _message(message) {}
    const char* what() const noexcept override { return _message.c_str(); }
};

// OpenCV-compatible single-channel type codes (CV_MAKETYPE(depth, 1)).
enum ImageType : int { U8 = 0, U16 = 2, S16 = 3, F32 = 5, F64 = 6 };

enum class Memory { Host, Device };

// Single-channel 2-D image in host or device memory. Copies share the pixels
// (like cv::Mat); create() (re)allocates owned storage; views wrap foreign memory.
class HipImage {
public:
    HipImage() = default;
    // Non-owning view over existing memory. step in bytes (0 = dense rows).
    HipImage(int rows, int cols, int type, void* data, size_t step = 0,
             Memory mem = Memory::Host);

    // Allocate owned storage (host: malloc'd, device: hipMalloc'd on the current device).
    void create(int rows, int cols, int type, Memory mem);
    static HipImage allocate(int rows, int cols, int type, Memory mem) {
        HipImage m;
        m.create(rows, cols, type, mem);
        return m;
    }

    void* data() const { return _data; }
    int rows() const { return _rows; }
    int cols() const { return _cols; }
    size_t step() const { return _step; }
    int type() const { return _type; }
    int depth() const { return _type; }
    size_t elemSize() const { return elem_size(_type); }
    Memory memory() const { return _mem; }
    bool empty() const { return _data == nullptr || _rows == 0 || _cols == 0; }

    template <typename T>
    T* ptr(int row) const {
        return reinterpret_cast<T*>(static_cast<char*>(_data) + (size_t)row * _step);
    }
    template <typename T>
    T& at(int row, int col) const {  // host memory only
        return ptr<T>(row)[col];
    }

    // Copy to host (returns *this when already on the host).
    HipImage download() const;

    static size_t elem_size(int type);

private:
    std::shared_ptr<void> _owner;
    void* _data = nullptr;
    int _rows = 0, _cols = 0, _type = U8;
    size_t _step = 0;
    Memory _mem = Memory::Host;
};

}  // namespace BICOS
