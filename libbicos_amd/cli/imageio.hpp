// imageio.hpp -- the file side of bicos-cli without OpenCV: what the reference gets from
// cv::imread / cv::imwrite / cv::normalize / cv::applyColorMap / cv::FileStorage /
// cv::reprojectImageTo3D (reference src/fileutils.cpp:30-154, include/fileutils.hpp:44-89,
// src/cli.cpp:228-250), on zlib alone:
//   * PNG decode (8/16-bit; gray, gray+alpha, RGB, RGBA, palette; 1/2/4-bit gray) and PGM
//     (P5) decode into single-channel U8 / U16 images;
//   * PNG encode (8-bit RGB), uncompressed TIFF encode (S16 / F32 / F64, one channel);
//   * min-max normalisation to 8 bits under a validity mask and the TURBO / VIRIDIS
//     colour maps (polynomial fits of the published maps: for viewing only);
//   * the stereo Q matrix from an OpenCV FileStorage file (YAML or XML) and the
//     disparity -> point reprojection with the .xyz writer.
#pragma once

#include <bicos/common.hpp>

#include <array>
#include <cstdint>
#include <optional>
#include <string>
#include <vector>

namespace bicos_cli {

// An owned single-channel host image (BICOS::Image view over `pixels`).
struct Gray {
    int rows = 0, cols = 0;
    int type = BICOS::U8;  // U8 or U16
    std::vector<uint8_t> pixels;
    BICOS::Image view() {
        return BICOS::Image(rows, cols, type, pixels.data(), 0, BICOS::Memory::Host);
    }
};

// Decode a PNG or binary PGM as one grey channel. keep16: keep 16-bit samples (the
// reference's IMREAD_ANYDEPTH); otherwise 16-bit samples are reduced to their high byte.
// Colour is converted like OpenCV's BGR2GRAY. Throws std::runtime_error.
Gray read_gray(const std::string& path, bool keep16);

// Decode PNG bytes (exposed for tests).
Gray decode_png(const std::vector<uint8_t>& bytes, bool keep16);

void write_png_rgb(const std::string& path, int rows, int cols, const std::vector<uint8_t>& rgb);
void write_png_gray8(const std::string& path, int rows, int cols, const std::vector<uint8_t>& g);
// One-channel TIFF of the image's own sample type (S16, F32, F64; also U8 / U16).
void write_tiff(const std::string& path, const BICOS::Image& img);

enum class Colormap { Turbo, Viridis };
// reference save_image (src/fileutils.cpp:30-58): min-max normalise the valid pixels to
// 0..255 (invalid = NaN for float maps, INVALID_DISP<int16_t> for S16), colour them, paint
// invalid pixels black; returns rows*cols*3 RGB bytes.
std::vector<uint8_t> colorize(const BICOS::Image& img, Colormap cmap);
std::array<uint8_t, 3> colormap_rgb(Colormap cmap, uint8_t v);

// The 4x4 matrix named `name` in an OpenCV FileStorage file (YAML "!!opencv-matrix" or XML
// type_id="opencv-matrix"), row-major.
std::array<double, 16> read_filestorage_matrix(const std::string& path, const std::string& name);

struct XyzStats {
    size_t written = 0, nonfinite = 0, negative_z = 0;
};
// cv::reprojectImageTo3D (handleMissingValues = false, float output) + the reference's
// save_pointcloud (include/fileutils.hpp:44-89): one "x y z" line per valid pixel.
XyzStats write_xyz(const std::string& path, const BICOS::Image& disparity,
                   const std::array<double, 16>& Q, bool allow_negative_z);

// reference read_sequence + sort_sequence_to_stack (src/fileutils.cpp:60-154): with two
// folders, files named <idx>.<ext> in each (16-bit kept); with one, <idx>_left.<ext> and
// <idx>_right.<ext> (8-bit). Sorted by index.
void read_stacks(const std::string& folder0, const std::optional<std::string>& folder1,
                 std::vector<Gray>& left, std::vector<Gray>& right);

}  // namespace bicos_cli
