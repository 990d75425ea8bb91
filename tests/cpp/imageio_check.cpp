// imageio_check.cpp -- TEST PROGRAM (tests/test_cli.py): exposes bicos-cli's file layer
// (libbicos_amd/cli/imageio.cpp) command by command so the Python tests can check it on
// the CPU against independent Python encoders/decoders.
//   decode IMG KEEP16 OUT        -> OUT: int32 rows, cols, type, then the pixels
//   tiff RAW ROWS COLS TYPE OUT  -> one-channel TIFF of the raw samples
//   colorize RAW ROWS COLS TYPE CMAP(0 turbo, 1 viridis) OUT -> rows*cols*3 RGB bytes
//   png RAW ROWS COLS OUT        -> 8-bit grey PNG
//   matrix FILE NAME             -> the 16 numbers on stdout
//   xyz RAW ROWS COLS TYPE QFILE ALLOWNEG OUT
#include <bicos/common.hpp>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <iterator>
#include <string>
#include <vector>

#include "../../libbicos_amd/cli/imageio.hpp"

using namespace bicos_cli;

static std::vector<uint8_t> slurp(const char* p) {
    std::ifstream f(p, std::ios::binary);
    return std::vector<uint8_t>(std::istreambuf_iterator<char>(f), {});
}

int main(int argc, char** argv) {
    try {
        const std::string cmd = argc > 1 ? argv[1] : "";
        if (cmd == "decode" && argc == 5) {
            Gray g = read_gray(argv[2], std::atoi(argv[3]) != 0);
            std::ofstream o(argv[4], std::ios::binary);
            const int hdr[3] = {g.rows, g.cols, g.type};
            o.write((const char*)hdr, sizeof hdr);
            o.write((const char*)g.pixels.data(), (std::streamsize)g.pixels.size());
            return 0;
        }
        if ((cmd == "tiff" || cmd == "colorize" || cmd == "xyz") && argc >= 7) {
            std::vector<uint8_t> raw = slurp(argv[2]);
            const BICOS::Image img(std::atoi(argv[3]), std::atoi(argv[4]), std::atoi(argv[5]),
                                   raw.data(), 0, BICOS::Memory::Host);
            if (cmd == "tiff") {
                write_tiff(argv[6], img);
                return 0;
            }
            if (cmd == "colorize" && argc == 8) {
                const auto rgb = colorize(img, std::atoi(argv[6]) ? Colormap::Viridis : Colormap::Turbo);
                std::ofstream(argv[7], std::ios::binary).write((const char*)rgb.data(), (std::streamsize)rgb.size());
                return 0;
            }
            if (cmd == "xyz" && argc == 9) {
                const auto st = write_xyz(argv[8], img, read_filestorage_matrix(argv[6], "Q"),
                                          std::atoi(argv[7]) != 0);
                std::printf("%zu %zu %zu\n", st.written, st.nonfinite, st.negative_z);
                return 0;
            }
        }
        if (cmd == "png" && argc == 6) {
            write_png_gray8(argv[5], std::atoi(argv[3]), std::atoi(argv[4]), slurp(argv[2]));
            return 0;
        }
        if (cmd == "matrix" && argc == 4) {
            for (double v : read_filestorage_matrix(argv[2], argv[3])) std::printf("%.17g\n", v);
            return 0;
        }
        std::cerr << "bad arguments\n";
        return 2;
    } catch (const std::exception& e) {
        std::cerr << "error: " << e.what() << std::endl;
        return 1;
    }
}
