// match_cpp.cpp -- TEST PROGRAM (tests/test_cpp_api.py, -m gpu): drives the C++ API the way a
// reference C++ caller does (reference include/match.hpp:31-41, src/lib.cpp:31-49) through
// every input branch of BICOS::match, and writes the maps for the Python test to compare
// with the CPU oracle:
//   host        host Images with padded rows (banded pinned upload path)
//   dev_planar  device Images that are views into ONE planar buffer per stack (zero-copy)
//   dev_staged  device Images in separate pitched allocations (2-D staging copies)
//   mats        an OpenCV-shaped matrix type through bicos/opencv.hpp's match_mats
//   seam        BICOS::impl::hip::match called directly (reference impl::cpu/cuda seam)
//
//   match_cpp <in.bin> <out_prefix> <nxcorr|-1> <subpixel|-1> <minvar|-1> <mode 0/1>
//             <variant 0/1> <max_lr_diff> <no_dupes> <precision 0/1>
// in.bin: int32 n, rows, cols, depth, then stack0 and stack1 as dense planes.
// Writes <out_prefix>.<branch>.disp / .corr (raw, dense) and one line per branch on stdout.
// the reference's installed header name (no OpenCV here: BICOS::Image = BICOS::HipImage)
#include <BICOS/match.hpp>
#include <bicos/opencv.hpp>
#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

using namespace BICOS;

static void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) {
        std::fprintf(stderr, "%s: %s\n", what, hipGetErrorString(e));
        std::exit(3);
    }
}

// minimal matrix type with the cv::Mat members match_mats uses (test double, host only)
struct TestMat {
    int rows = 0, cols = 0;
    unsigned char* data = nullptr;
    size_t step[2] = {0, 0};
    int t = 0;
    std::vector<unsigned char> buf;
    int type() const { return t; }
    void create(int r, int c, int ty) {
        rows = r;
        cols = c;
        t = ty;
        step[1] = Image::elem_size(ty);
        step[0] = (size_t)c * step[1];
        buf.assign(step[0] * r, 0);
        data = buf.data();
    }
};

static void write_out(const std::string& path, const Image& m) {
    Image h = m.download();
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) std::exit(4);
    const size_t row = (size_t)h.cols() * h.elemSize();
    for (int r = 0; r < h.rows(); ++r) std::fwrite(h.ptr<char>(r), 1, row, f);
    std::fclose(f);
}

int main(int argc, char** argv) {
    if (argc != 11) {
        std::fprintf(stderr, "usage: see header\n");
        return 2;
    }
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    int hdr[4];
    if (std::fread(hdr, sizeof(int), 4, f) != 4) return 2;
    const int n = hdr[0], rows = hdr[1], cols = hdr[2], depth = hdr[3];
    const size_t plane = (size_t)rows * cols * depth;
    std::vector<unsigned char> raw(2 * n * plane);
    if (std::fread(raw.data(), 1, raw.size(), f) != raw.size()) return 2;
    std::fclose(f);
    const std::string out = argv[2];

    Config cfg;
    const float nxc = std::atof(argv[3]), sub = std::atof(argv[4]), mv = std::atof(argv[5]);
    cfg.nxcorr_threshold = nxc >= 0 ? std::optional<float>(nxc) : std::nullopt;
    if (sub > 0) cfg.subpixel_step = sub;
    if (mv >= 0) cfg.min_variance = mv;
    cfg.mode = std::atoi(argv[6]) ? TransformMode::FULL : TransformMode::LIMITED;
    if (std::atoi(argv[7])) cfg.variant = Variant::Consistency{std::atoi(argv[8]), std::atoi(argv[9]) != 0};
    cfg.precision = std::atoi(argv[10]) ? Precision::DOUBLE : Precision::SINGLE;
    const int type = depth == 1 ? U8 : U16;
    const size_t rowb = (size_t)cols * depth;
    auto src = [&](int s, int t) { return raw.data() + ((size_t)s * n + t) * plane; };

    auto report = [&](const char* name, const Image& d, const Image& c) {
        write_out(out + "." + name + ".disp", d);
        if (!c.empty()) write_out(out + "." + name + ".corr", c);
        std::printf("%s type=%d corr_type=%d rows=%d cols=%d mem=%s\n", name, d.type(),
                    c.empty() ? -1 : c.type(), d.rows(), d.cols(),
                    d.memory() == Memory::Host ? "host" : "device");
    };

    // optional MATCH_CPP_ORDER=b1,b2,... runs only those branches, in that order (debugging)
    const char* order_env = std::getenv("MATCH_CPP_ORDER");
    const std::string order = order_env ? order_env : "host,dev_planar,dev_staged,mats,seam";
    hipStream_t st;
    hip_ok(hipStreamCreate(&st), "hipStreamCreate");
    auto run_host = [&]() {
        const size_t step = rowb + 13 * depth;
        std::vector<std::vector<unsigned char>> keep;
        std::vector<Image> s0, s1;
        for (int s = 0; s < 2; ++s)
            for (int t = 0; t < n; ++t) {
                keep.emplace_back(step * rows);
                for (int r = 0; r < rows; ++r)
                    std::memcpy(keep.back().data() + r * step, src(s, t) + r * rowb, rowb);
                (s ? s1 : s0).emplace_back(rows, cols, type, keep.back().data(), step, Memory::Host);
            }
        Image d, c;
        match(s0, s1, d, cfg, &c);
        report("host", d, c);
    };
    // 2. device, one planar buffer per stack (pitch cols + 64 elements, planes 3 rows apart
    //    more than needed): the zero-copy branch
    auto run_planar = [&]() {
        const size_t step = rowb + 64 * depth, pstride = step * (rows + 3);
        std::vector<Image> s0, s1;
        void* buf[2];
        for (int s = 0; s < 2; ++s) {
            hip_ok(hipMalloc(&buf[s], pstride * n), "hipMalloc");
            for (int t = 0; t < n; ++t) {
                char* p = (char*)buf[s] + t * pstride;
                hip_ok(hipMemcpy2D(p, step, src(s, t), rowb, rowb, rows, hipMemcpyHostToDevice), "upload");
                (s ? s1 : s0).emplace_back(rows, cols, type, p, step, Memory::Device);
            }
        }
        Image d, c;
        match(s0, s1, d, cfg, &c, st);
        hip_ok(hipStreamSynchronize(st), "sync");
        report("dev_planar", d, c);
        hip_ok(hipFree(buf[0]), "free");
        hip_ok(hipFree(buf[1]), "free");
    };
    // 3. device, separate pitched allocations: the staging branch
    auto run_staged = [&]() {
        std::vector<Image> s0, s1;
        std::vector<void*> bufs;
        for (int s = 0; s < 2; ++s)
            for (int t = 0; t < n; ++t) {
                void* p;
                size_t pitch;
                hip_ok(hipMallocPitch(&p, &pitch, rowb + 5, rows), "hipMallocPitch");
                bufs.push_back(p);
                hip_ok(hipMemcpy2D(p, pitch, src(s, t), rowb, rowb, rows, hipMemcpyHostToDevice), "upload");
                (s ? s1 : s0).emplace_back(rows, cols, type, p, pitch, Memory::Device);
                std::vector<unsigned char> back(plane);
                hip_ok(hipMemcpy2D(back.data(), rowb, p, pitch, rowb, rows, hipMemcpyDeviceToHost), "check");
                if (std::memcmp(back.data(), src(s, t), plane)) {
                    std::fprintf(stderr, "upload of stack %d plane %d differs\n", s, t);
                    std::exit(5);
                }
            }
        Image d, c;
        match(s0, s1, d, cfg, &c, st);
        hip_ok(hipStreamSynchronize(st), "sync");
        report("dev_staged", d, c);
        for (void* p : bufs) hip_ok(hipFree(p), "free");
    };
    // 4. OpenCV-shaped matrices through bicos/opencv.hpp
    auto run_mats = [&]() {
        std::vector<TestMat> m0(n), m1(n);
        for (int t = 0; t < n; ++t) {
            m0[t].create(rows, cols, type);
            m1[t].create(rows, cols, type);
            std::memcpy(m0[t].data, src(0, t), plane);
            std::memcpy(m1[t].data, src(1, t), plane);
        }
        TestMat d, c;
        match_mats(m0, m1, d, cfg, &c);
        report("mats", image_view(d), c.data ? image_view(c) : Image());
    };
    // 5. the backend seam directly, host images without padding
    auto run_seam = [&]() {
        std::vector<Image> s0, s1;
        for (int t = 0; t < n; ++t) {
            s0.emplace_back(rows, cols, type, src(0, t), 0, Memory::Host);
            s1.emplace_back(rows, cols, type, src(1, t), 0, Memory::Host);
        }
        Image d, c;
        impl::hip::match(s0, s1, d, cfg, &c, nullptr);
        report("seam", d, c);
    };
    size_t pos = 0;
    while (pos <= order.size()) {
        size_t e = order.find(',', pos);
        if (e == std::string::npos) e = order.size();
        const std::string b = order.substr(pos, e - pos);
        if (b == "host") run_host();
        else if (b == "dev_planar") run_planar();
        else if (b == "dev_staged") run_staged();
        else if (b == "mats") run_mats();
        else if (b == "seam") run_seam();
        pos = e + 1;
    }
    // errors surface as BICOS::Exception, as in the reference
    try {
        std::vector<Image> one(1, Image(rows, cols, type, src(0, 0), 0, Memory::Host));
        Image d;
        match(one, one, d, cfg);
        std::printf("error_case none\n");
    } catch (const Exception& e) {
        std::printf("error_case %s\n", e.what());
    }
    hip_ok(hipStreamDestroy(st), "hipStreamDestroy");
    return 0;
}
