// bicos-cli -- the reference's command-line front end (reference src/cli.cpp:55-253) on the
// gfx950 engine, without OpenCV, cxxopts or fmt: a folder of numbered images in (PNG or
// binary PGM), the disparity out as a colourised PNG plus the raw map as TIFF, optionally
// the correlation map and a point cloud (.xyz) through a stereo Q matrix.
//
//   bicos-cli folder0 [folder1] [-t 0.75] [-v VAR] [-s STEP] [-o bicosdisp.png] [-n N]
//             [-q Q.yml] [--allow-negative-z] [-m MAXDIFF] [--double] [--limited]
//             [--corrmap] [--no-dupes] [-h]
//
// Same options, defaults and semantics as the reference (FULL transform unless --limited;
// --threshold <= 0 disables the NXC filter; --corrmap without a threshold computes with
// threshold -1; the variance filter only when -v is given and > 0; --lr-maxdiff selects
// the Consistency variant, --no-dupes then adds duplicate rejection). Divergence: the
// reference declares --allow-negative-z but reads "allow-behind" (cli.cpp:233), so its flag
// never takes effect; here it does.
#include <bicos/common.hpp>
#include <bicos/match.hpp>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <filesystem>
#include <iostream>
#include <map>
#include <optional>
#include <string>
#include <unistd.h>
#include <vector>

#include "imageio.hpp"

using namespace BICOS;
namespace fs = std::filesystem;

namespace {

const char* USAGE =
    "bicos-cli: process multi-shot stereo images with BICOS (libbicos_amd, gfx950)\n"
    "usage: bicos-cli folder0 [folder1] [options]\n"
    "  folder0                 first folder with numbered input images\n"
    "  folder1                 optional second folder; then names are 0.png, 1.png...\n"
    "                          else folder0 holds 0_left.png, 0_right.png, 1_left.png...\n"
    "  -t, --threshold F       minimum normalized cross correlation of a match (0.75;\n"
    "                          0.0 disables)\n"
    "  -v, --variance F        minimum intensity variance (only with --threshold)\n"
    "  -s, --step F            subpixel interpolation step (only with --threshold)\n"
    "  -o, --out FILE          output file for the disparity image (bicosdisp.png)\n"
    "  -n, --stacksize N       number of images to process (default: all found)\n"
    "  -q, --qmatrix FILE      OpenCV FileStorage (YAML/XML) with a 4x4 matrix \"Q\":\n"
    "                          also write a point cloud (.xyz)\n"
    "      --allow-negative-z  keep points with negative Z in the point cloud\n"
    "  -m, --lr-maxdiff N      maximum left-right disparity difference (Consistency\n"
    "                          variant; disables duplicate filtering)\n"
    "      --double            double precision correlation\n"
    "      --limited           LIMITED transform mode (allows more images)\n"
    "      --corrmap           also write the map of correlation values\n"
    "      --no-dupes          duplicate filtering (the default without --lr-maxdiff)\n"
    "  -h, --help              this message\n";

struct Args {
    std::vector<std::string> pos;
    std::map<std::string, std::string> val;  // option -> value ("" for flags)
    bool has(const std::string& k) const { return val.count(k) != 0; }
};

Args parse(int argc, char** argv) {
    static const std::map<std::string, std::string> shorts = {
        {"t", "threshold"}, {"v", "variance"}, {"s", "step"}, {"o", "out"},
        {"n", "stacksize"}, {"q", "qmatrix"}, {"m", "lr-maxdiff"}, {"h", "help"}};
    static const std::map<std::string, bool> takes = {
        {"threshold", true}, {"variance", true}, {"step", true}, {"out", true},
        {"stacksize", true}, {"qmatrix", true}, {"lr-maxdiff", true}, {"help", false},
        {"allow-negative-z", false}, {"double", false}, {"limited", false},
        {"corrmap", false}, {"no-dupes", false}};
    Args a;
    for (int i = 1; i < argc; ++i) {
        std::string s = argv[i];
        if (s.size() < 2 || s[0] != '-') {
            a.pos.push_back(s);
            continue;
        }
        std::string name, value;
        bool inline_value = false;
        if (s[1] == '-') {
            name = s.substr(2);
            const size_t eq = name.find('=');
            if (eq != std::string::npos) {
                value = name.substr(eq + 1);
                name = name.substr(0, eq);
                inline_value = true;
            }
        } else {
            const auto it = shorts.find(s.substr(1, 1));
            if (it == shorts.end()) throw std::invalid_argument("unknown option " + s);
            name = it->second;
            if (s.size() > 2) value = s.substr(2), inline_value = true;
        }
        const auto t = takes.find(name);
        if (t == takes.end()) throw std::invalid_argument("unknown option --" + name);
        if (t->second && !inline_value) {
            if (i + 1 >= argc) throw std::invalid_argument("option --" + name + " needs a value");
            value = argv[++i];
        }
        a.val[name] = value;
    }
    return a;
}

float as_float(const Args& a, const std::string& k) {
    size_t used = 0;
    const float v = std::stof(a.val.at(k), &used);
    if (used != a.val.at(k).size()) throw std::invalid_argument("--" + k + ": not a number");
    return v;
}

unsigned as_uint(const Args& a, const std::string& k) {
    const std::string& s = a.val.at(k);
    if (s.empty() || s.find_first_not_of("0123456789") != std::string::npos)
        throw std::invalid_argument("--" + k + ": not an unsigned integer");
    return (unsigned)std::stoul(s);
}

double ms_since(std::chrono::high_resolution_clock::time_point t) {
    return std::chrono::duration_cast<std::chrono::microseconds>(
               std::chrono::high_resolution_clock::now() - t).count() / 1000.0;
}

// reference save_image (src/fileutils.cpp:30-58): colourised PNG and raw TIFF
void save_image(const Image& img, fs::path out, bicos_cli::Colormap cmap) {
    const std::vector<uint8_t> rgb = bicos_cli::colorize(img, cmap);
    bicos_cli::write_png_rgb(out.replace_extension("png").string(), img.rows(), img.cols(), rgb);
    std::cout << "Saved colorized disparity to\t\t" << out << std::endl;
    bicos_cli::write_tiff(out.replace_extension("tiff").string(), img);
    std::cout << "Saved floating-point disparity to\t" << out << std::endl;
}

int run(int argc, char** argv) {
    const Args args = parse(argc, argv);
    if (args.has("help") || args.pos.empty()) {
        std::cout << USAGE;
        return args.has("help") ? 0 : 2;
    }
    if (args.pos.size() > 2) throw std::invalid_argument("at most two input folders");
    std::cout << "bicos-cli (libbicos_amd: BICOS on the MI355X)\n" << std::endl;
    if (!isatty(STDOUT_FILENO)) std::cerr << "Danger: bicos-cli does not have a stable CLI interface\n";
    if (args.has("no-dupes") && !args.has("lr-maxdiff"))
        std::cerr << "'no-dupes' is the default when 'lr-maxdiff' is not set.\n";

    const std::string folder0 = args.pos[0];
    const fs::path outfile = args.has("out") ? args.val.at("out") : "bicosdisp.png";
    std::optional<std::string> folder1;
    if (args.pos.size() == 2) folder1 = args.pos[1];
    std::optional<std::string> q_store;
    if (args.has("qmatrix")) {
        q_store = args.val.at("qmatrix");
        if (!fs::exists(*q_store)) throw std::invalid_argument("'" + *q_store + "' does not exist");
    }

    std::vector<bicos_cli::Gray> left, right;
    bicos_cli::read_stacks(folder0, folder1, left, right);
    if (args.has("stacksize")) {
        const unsigned n = as_uint(args, "stacksize");
        if (n < left.size()) {
            left.resize(n);
            right.resize(n);
        }
    }
    if (left.empty()) throw std::invalid_argument("no input images");
    std::cout << "Loaded " << left.size() + right.size() << " "
              << (left.front().type == U16 ? 16 : 8) << "-bit images in total" << std::endl;

    Config c;
    c.nxcorr_threshold = args.has("threshold") ? as_float(args, "threshold") : 0.75f;
    c.mode = TransformMode::FULL;
    if (*c.nxcorr_threshold <= 0.0f) c.nxcorr_threshold = std::nullopt;
    const bool need_corrmap = args.has("corrmap");
    if (need_corrmap && !c.nxcorr_threshold) {
        c.nxcorr_threshold = -1.0f;
        std::cerr << "Computing with nxcorr-threshold of -1 because 'corrmap' is set\n";
    }
    if (args.has("step")) c.subpixel_step = as_float(args, "step");
    if (args.has("limited")) c.mode = TransformMode::LIMITED;
    if (args.has("variance"))
        if (const float mv = as_float(args, "variance"); mv > 0.0f) c.min_variance = mv;
    if (args.has("double")) c.precision = Precision::DOUBLE;
    if (args.has("lr-maxdiff"))
        c.variant = Variant::Consistency{(int)as_uint(args, "lr-maxdiff"), args.has("no-dupes")};

    std::vector<Image> s0, s1;
    for (auto& g : left) s0.push_back(g.view());
    for (auto& g : right) s1.push_back(g.view());
    Image disp, corrmap;
    const auto tick = std::chrono::high_resolution_clock::now();
    BICOS::match(s0, s1, disp, c, need_corrmap ? &corrmap : nullptr);
    std::cout << "Latency:\t" << ms_since(tick) << "ms" << std::endl;

    save_image(disp, outfile, bicos_cli::Colormap::Turbo);
    if (need_corrmap)
        save_image(corrmap,
                   outfile.parent_path() /
                       (outfile.stem().string() + "-corrmap" + outfile.extension().string()),
                   bicos_cli::Colormap::Viridis);

    if (q_store) {
        const auto Q = bicos_cli::read_filestorage_matrix(*q_store, "Q");
        fs::path xyz = outfile;
        xyz.replace_extension("xyz");
        const auto st = bicos_cli::write_xyz(xyz.string(), disp, Q, args.has("allow-negative-z"));
        std::cout << "Saved pointcloud in ascii-format to\t" << xyz << std::endl;
        if (st.nonfinite) std::cerr << "Skipped " << st.nonfinite << " points with non-finite fp values" << std::endl;
        if (st.negative_z) std::cerr << "Skipped " << st.negative_z << " points with negative Z values" << std::endl;
    }
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    try {
        return run(argc, argv);
    } catch (const std::exception& e) {
        std::cerr << "bicos-cli: " << e.what() << std::endl;
        return 1;
    }
}
