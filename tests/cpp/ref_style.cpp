// ref_style.cpp -- TEST PROGRAM (tests/test_cpp_api.py): a translation unit written the way a
// reference libBICOS C++ caller writes it -- `#include <BICOS/match.hpp>`, `BICOS::Image`
// maps, std::vector<cv::Mat> stacks, BICOS::Config with a Variant, BICOS::match(stack0,
// stack1, disparity, cfg, &corrmap), BICOS::is_invalid / INVALID_DISP, BICOS::Exception
// (reference include/match.hpp:31-41, include/common.hpp:34-90) -- built against the
// INSTALLED tree (find_package(BICOS), tests/cpp/consumer/CMakeLists.txt) with nothing but
// the reference's names. OpenCV is absent here, so cv::Mat comes from the test double in
// tests/cpp/cvmat_double/.
//
//   ref_style <in.bin> <out_prefix> <nxcorr|-1> <subpixel|-1> <minvar|-1> <limited 0/1>
//             <consistency 0/1> <max_lr_diff> <no_dupes>
// in.bin: int32 n, rows, cols, depth, then stack0 and stack1 as dense planes (match_cpp's
// format). Writes <out_prefix>.ref.disp / .corr and one summary line.
#include <BICOS/match.hpp>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#ifndef BICOS_IMAGE_IS_CV_MAT
#error "expected BICOS::Image = cv::Mat (the reference CPU build's Image)"
#endif

int main(int argc, char** argv) {
    if (argc != 10) {
        std::fprintf(stderr, "usage: ref_style in.bin out_prefix nxcorr subpix minvar limited "
                             "consistency max_lr_diff no_dupes\n");
        return 2;
    }
    FILE* f = std::fopen(argv[1], "rb");
    int hdr[4];
    if (!f || std::fread(hdr, sizeof(int), 4, f) != 4) return 2;
    const int n = hdr[0], rows = hdr[1], cols = hdr[2], depth = hdr[3];
    const int type = depth == 1 ? CV_8UC1 : CV_16UC1;
    std::vector<BICOS::Image> stack0, stack1;
    for (int s = 0; s < 2; ++s)
        for (int t = 0; t < n; ++t) {
            cv::Mat m(rows, cols, type);
            if (std::fread(m.data, (size_t)depth * cols, rows, f) != (size_t)rows) return 2;
            (s ? stack1 : stack0).push_back(m);
        }
    std::fclose(f);

    BICOS::Config cfg;
    const float nxc = std::atof(argv[3]), sp = std::atof(argv[4]), mv = std::atof(argv[5]);
    cfg.nxcorr_threshold = nxc < 0 ? std::nullopt : std::optional<float>(nxc);
    if (sp > 0) cfg.subpixel_step = sp;
    if (mv >= 0) cfg.min_variance = mv;
    cfg.mode = std::atoi(argv[6]) ? BICOS::TransformMode::LIMITED : BICOS::TransformMode::FULL;
    if (std::atoi(argv[7]))
        cfg.variant = BICOS::Variant::Consistency{std::atoi(argv[8]), std::atoi(argv[9]) != 0};
    else
        cfg.variant = BICOS::Variant::NoDuplicates{};

    BICOS::Image disparity, corrmap;
    try {
        BICOS::match(stack0, stack1, disparity, cfg, &corrmap);
    } catch (const BICOS::Exception& e) {
        std::printf("exception: %s\n", e.what());
        return 5;
    }
    long invalid = 0;
    for (int r = 0; r < disparity.rows; ++r)
        for (int c = 0; c < disparity.cols; ++c) {
            if (disparity.type() == CV_16S)
                invalid += BICOS::is_invalid(disparity.at<int16_t>(r, c));
            else if (cfg.subpixel_step)
                invalid += BICOS::is_invalid(disparity.at<float>(r, c));
            else
                invalid += disparity.at<float>(r, c) == (float)BICOS::INVALID_DISP<int16_t>;
        }
    const std::string out = argv[2];
    FILE* o = std::fopen((out + ".ref.disp").c_str(), "wb");
    std::fwrite(disparity.data, disparity.step[0], disparity.rows, o);
    std::fclose(o);
    if (!corrmap.empty()) {
        o = std::fopen((out + ".ref.corr").c_str(), "wb");
        std::fwrite(corrmap.data, corrmap.step[0], corrmap.rows, o);
        std::fclose(o);
    }
    std::printf("ref_style %s type=%d invalid=%ld corr=%d\n", BICOS_VERSION, disparity.type(),
                invalid, corrmap.empty() ? 0 : corrmap.type());
    return 0;
}
