// imageio.cpp -- see imageio.hpp. Host code only (zlib + the C++ standard library).
#include "imageio.hpp"

#include <zlib.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <iterator>
#include <sstream>
#include <stdexcept>

namespace bicos_cli {

namespace {

std::vector<uint8_t> slurp(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open " + path);
    return std::vector<uint8_t>(std::istreambuf_iterator<char>(f), {});
}

uint32_t be32(const uint8_t* p) {
    return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}

void put_be32(std::vector<uint8_t>& v, uint32_t x) {
    for (int s = 24; s >= 0; s -= 8) v.push_back((uint8_t)(x >> s));
}

// libpng's png_set_rgb_to_gray(png, 1, 0.299, 0.587) -- OpenCV's PNG reader for
// IMREAD_GRAYSCALE: coefficients in 1/32768 units, rounded
uint32_t rgb_to_gray(uint32_t r, uint32_t g, uint32_t b) {
    return (9798u * r + 19235u * g + 3735u * b + 16384u) >> 15;
}

uint8_t paeth(int a, int b, int c) {
    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    if (pa <= pb && pa <= pc) return (uint8_t)a;
    return (uint8_t)(pb <= pc ? b : c);
}

Gray decode_pgm(const std::vector<uint8_t>& b, bool keep16) {
    size_t i = 2;
    auto token = [&]() {
        for (;;) {
            while (i < b.size() && std::isspace(b[i])) ++i;
            if (i < b.size() && b[i] == '#') {
                while (i < b.size() && b[i] != '\n') ++i;
                continue;
            }
            break;
        }
        long v = 0;
        size_t start = i;
        while (i < b.size() && std::isdigit(b[i])) v = v * 10 + (b[i++] - '0');
        if (i == start) throw std::runtime_error("malformed PGM header");
        return v;
    };
    const long w = token(), h = token(), maxval = token();
    ++i;  // the single whitespace before the raster
    if (w <= 0 || h <= 0 || maxval <= 0 || maxval > 65535) throw std::runtime_error("bad PGM");
    const int bps = maxval < 256 ? 1 : 2;
    if (b.size() < i + (size_t)w * h * bps) throw std::runtime_error("truncated PGM");
    Gray g;
    g.rows = (int)h;
    g.cols = (int)w;
    g.type = bps == 2 && keep16 ? BICOS::U16 : BICOS::U8;
    g.pixels.resize((size_t)w * h * (g.type == BICOS::U16 ? 2 : 1));
    for (size_t k = 0; k < (size_t)w * h; ++k) {
        const uint32_t v = bps == 1 ? b[i + k] : (uint32_t)b[i + 2 * k] << 8 | b[i + 2 * k + 1];
        if (g.type == BICOS::U16)
            reinterpret_cast<uint16_t*>(g.pixels.data())[k] = (uint16_t)v;
        else
            g.pixels[k] = (uint8_t)(bps == 2 ? v >> 8 : v);
    }
    return g;
}

uint32_t png_crc(const char* type, const uint8_t* data, size_t n) {
    uLong c = crc32(0L, Z_NULL, 0);
    c = crc32(c, reinterpret_cast<const Bytef*>(type), 4);
    if (n) c = crc32(c, data, (uInt)n);
    return (uint32_t)c;
}

void png_chunk(std::vector<uint8_t>& out, const char* type, const std::vector<uint8_t>& data) {
    put_be32(out, (uint32_t)data.size());
    out.insert(out.end(), type, type + 4);
    out.insert(out.end(), data.begin(), data.end());
    put_be32(out, png_crc(type, data.data(), data.size()));
}

void write_png(const std::string& path, int rows, int cols, int channels,
               const std::vector<uint8_t>& px) {
    std::vector<uint8_t> raw;
    raw.reserve((size_t)rows * (cols * channels + 1));
    for (int r = 0; r < rows; ++r) {
        raw.push_back(0);  // filter: none
        const uint8_t* row = px.data() + (size_t)r * cols * channels;
        raw.insert(raw.end(), row, row + (size_t)cols * channels);
    }
    uLongf zlen = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK)
        throw std::runtime_error("zlib compression failed");
    z.resize(zlen);
    std::vector<uint8_t> out = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
    std::vector<uint8_t> ihdr;
    put_be32(ihdr, (uint32_t)cols);
    put_be32(ihdr, (uint32_t)rows);
    ihdr.push_back(8);
    ihdr.push_back(channels == 3 ? 2 : 0);
    ihdr.push_back(0);
    ihdr.push_back(0);
    ihdr.push_back(0);
    png_chunk(out, "IHDR", ihdr);
    png_chunk(out, "IDAT", z);
    png_chunk(out, "IEND", {});
    std::ofstream f(path, std::ios::binary);
    if (!f.write(reinterpret_cast<const char*>(out.data()), (std::streamsize)out.size()))
        throw std::runtime_error("cannot write " + path);
}

double pixel(const BICOS::Image& m, int r, int c) {
    switch (m.type()) {
        case BICOS::U8: return m.at<uint8_t>(r, c);
        case BICOS::U16: return m.at<uint16_t>(r, c);
        case BICOS::S16: return m.at<int16_t>(r, c);
        case BICOS::F32: return m.at<float>(r, c);
        case BICOS::F64: return m.at<double>(r, c);
    }
    throw std::runtime_error("unsupported image type");
}

bool valid(const BICOS::Image& m, double v) {
    if (m.type() == BICOS::F32 || m.type() == BICOS::F64) return !std::isnan(v);
    return v != (double)BICOS::INVALID_DISP<int16_t>;
}

// the numbers of the first "[...]" (YAML) or "<data>...</data>" (XML) after position `at`
std::vector<double> numbers_after(const std::string& s, size_t at, bool xml) {
    size_t b = xml ? s.find("<data>", at) : s.find('[', s.find("data", at));
    if (b == std::string::npos) throw std::runtime_error("matrix has no data");
    b += xml ? 6 : 1;
    const size_t e = s.find(xml ? "</data>" : "]", b);
    if (e == std::string::npos) throw std::runtime_error("unterminated matrix data");
    std::string body = s.substr(b, e - b);
    std::replace(body.begin(), body.end(), ',', ' ');
    std::istringstream in(body);
    std::vector<double> v;
    double x;
    while (in >> x) v.push_back(x);
    return v;
}

}  // namespace

Gray decode_png(const std::vector<uint8_t>& b, bool keep16) {
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
    if (b.size() < 8 || std::memcmp(b.data(), sig, 8)) throw std::runtime_error("not a PNG");
    uint32_t w = 0, h = 0;
    int depth = 0, ctype = -1, interlace = 0;
    std::vector<uint8_t> idat, plte;
    for (size_t p = 8; p + 12 <= b.size();) {
        const uint32_t len = be32(&b[p]);
        if (p + 12 + (size_t)len > b.size()) throw std::runtime_error("truncated PNG chunk");
        const char* type = reinterpret_cast<const char*>(&b[p + 4]);
        const uint8_t* d = &b[p + 8];
        if (png_crc(type, d, len) != be32(d + len)) throw std::runtime_error("PNG CRC mismatch");
        if (!std::memcmp(type, "IHDR", 4)) {
            if (len < 13) throw std::runtime_error("bad IHDR");
            w = be32(d);
            h = be32(d + 4);
            depth = d[8];
            ctype = d[9];
            interlace = d[12];
        } else if (!std::memcmp(type, "PLTE", 4)) {
            plte.assign(d, d + len);
        } else if (!std::memcmp(type, "IDAT", 4)) {
            idat.insert(idat.end(), d, d + len);
        } else if (!std::memcmp(type, "IEND", 4)) {
            break;
        }
        p += 12 + (size_t)len;
    }
    if (!w || !h || w > (1u << 24) || h > (1u << 24)) throw std::runtime_error("bad PNG size");
    if (interlace) throw std::runtime_error("interlaced PNG is not supported");
    int ch;
    switch (ctype) {
        case 0: ch = 1; break;
        case 2: ch = 3; break;
        case 3: ch = 1; break;
        case 4: ch = 2; break;
        case 6: ch = 4; break;
        default: throw std::runtime_error("bad PNG colour type");
    }
    const bool ok_depth = depth == 8 || depth == 16 || ((ctype == 0 || ctype == 3) && depth < 8 &&
                                                         (depth == 1 || depth == 2 || depth == 4));
    if (!ok_depth || (ctype == 3 && depth == 16)) throw std::runtime_error("bad PNG bit depth");
    const size_t bits = (size_t)ch * depth;
    const size_t rowbytes = (w * bits + 7) / 8;
    const size_t bpp = std::max<size_t>(1, bits / 8);
    std::vector<uint8_t> raw(h * (rowbytes + 1));
    uLongf rlen = (uLongf)raw.size();
    if (uncompress(raw.data(), &rlen, idat.data(), (uLong)idat.size()) != Z_OK || rlen != raw.size())
        throw std::runtime_error("corrupt PNG image data");
    // unfilter in place (rows of rowbytes after a filter byte)
    std::vector<uint8_t> img(h * rowbytes);
    for (uint32_t r = 0; r < h; ++r) {
        const uint8_t f = raw[r * (rowbytes + 1)];
        const uint8_t* src = &raw[r * (rowbytes + 1) + 1];
        uint8_t* cur = &img[r * rowbytes];
        const uint8_t* up = r ? &img[(r - 1) * rowbytes] : nullptr;
        for (size_t i = 0; i < rowbytes; ++i) {
            const int a = i >= bpp ? cur[i - bpp] : 0, u = up ? up[i] : 0;
            const int c = up && i >= bpp ? up[i - bpp] : 0;
            int v = src[i];
            switch (f) {
                case 0: break;
                case 1: v += a; break;
                case 2: v += u; break;
                case 3: v += (a + u) / 2; break;
                case 4: v += paeth(a, u, c); break;
                default: throw std::runtime_error("bad PNG filter");
            }
            cur[i] = (uint8_t)v;
        }
    }
    Gray g;
    g.rows = (int)h;
    g.cols = (int)w;
    const bool out16 = depth == 16 && keep16;
    g.type = out16 ? BICOS::U16 : BICOS::U8;
    g.pixels.resize((size_t)w * h * (out16 ? 2 : 1));
    uint16_t* o16 = reinterpret_cast<uint16_t*>(g.pixels.data());
    for (uint32_t r = 0; r < h; ++r) {
        const uint8_t* row = &img[r * rowbytes];
        for (uint32_t c = 0; c < w; ++c) {
            // sample k of pixel c; 16-bit samples are reduced to their high byte unless kept
            auto sample = [&](int k) -> uint32_t {
                if (depth == 16) {
                    const uint32_t v = (uint32_t)row[(c * ch + k) * 2] << 8 | row[(c * ch + k) * 2 + 1];
                    return out16 ? v : v >> 8;
                }
                if (depth == 8) return row[c * ch + k];
                const size_t bit = (size_t)c * depth;  // 1/2/4-bit grey or palette index
                return (row[bit / 8] >> (8 - depth - bit % 8)) & ((1u << depth) - 1);
            };
            uint32_t v;
            if (ctype == 0 || ctype == 4) {
                v = sample(0);
                if (depth < 8) v = v * 255u / ((1u << depth) - 1);
            } else if (ctype == 3) {
                const uint32_t idx = sample(0);
                if (3 * idx + 2 >= plte.size()) throw std::runtime_error("PNG palette index out of range");
                v = rgb_to_gray(plte[3 * idx], plte[3 * idx + 1], plte[3 * idx + 2]);
            } else {
                v = rgb_to_gray(sample(0), sample(1), sample(2));
            }
            const size_t k = (size_t)r * w + c;
            if (out16)
                o16[k] = (uint16_t)v;
            else
                g.pixels[k] = (uint8_t)v;
        }
    }
    return g;
}

Gray read_gray(const std::string& path, bool keep16) {
    const std::vector<uint8_t> b = slurp(path);
    if (b.size() >= 8 && b[0] == 0x89 && b[1] == 'P' && b[2] == 'N' && b[3] == 'G')
        return decode_png(b, keep16);
    if (b.size() >= 2 && b[0] == 'P' && b[1] == '5') return decode_pgm(b, keep16);
    throw std::runtime_error(path + ": unsupported image format (PNG or binary PGM expected)");
}

void write_png_rgb(const std::string& path, int rows, int cols, const std::vector<uint8_t>& rgb) {
    write_png(path, rows, cols, 3, rgb);
}

void write_png_gray8(const std::string& path, int rows, int cols, const std::vector<uint8_t>& g) {
    write_png(path, rows, cols, 1, g);
}

void write_tiff(const std::string& path, const BICOS::Image& img) {
    int bits, format;  // SampleFormat: 1 unsigned, 2 signed, 3 IEEE float
    switch (img.type()) {
        case BICOS::U8: bits = 8, format = 1; break;
        case BICOS::U16: bits = 16, format = 1; break;
        case BICOS::S16: bits = 16, format = 2; break;
        case BICOS::F32: bits = 32, format = 3; break;
        case BICOS::F64: bits = 64, format = 3; break;
        default: throw std::runtime_error("unsupported TIFF sample type");
    }
    const uint32_t rows = (uint32_t)img.rows(), cols = (uint32_t)img.cols();
    const uint32_t rowb = cols * (uint32_t)bits / 8, bytes = rowb * rows;
    struct Entry {
        uint16_t tag, type;  // type 3 SHORT, 4 LONG
        uint32_t value;
    };
    const uint16_t ne = 11;
    const uint32_t data_off = 8 + 2 + ne * 12 + 4;
    const Entry e[ne] = {{256, 4, cols},     {257, 4, rows},        {258, 3, (uint32_t)bits},
                         {259, 3, 1},        {262, 3, 1},           {273, 4, data_off},
                         {277, 3, 1},        {278, 4, rows},        {279, 4, bytes},
                         {284, 3, 1},        {339, 3, (uint32_t)format}};
    std::vector<uint8_t> out;
    auto le16 = [&](uint16_t x) { out.push_back(x & 0xFF), out.push_back(x >> 8); };
    auto le32 = [&](uint32_t x) { for (int s = 0; s < 32; s += 8) out.push_back((uint8_t)(x >> s)); };
    out.push_back('I');
    out.push_back('I');
    le16(42);
    le32(8);
    le16(ne);
    for (const Entry& x : e) {
        le16(x.tag);
        le16(x.type);
        le32(1);
        if (x.type == 3) {
            le16((uint16_t)x.value);
            le16(0);
        } else {
            le32(x.value);
        }
    }
    le32(0);  // no further IFD
    for (uint32_t r = 0; r < rows; ++r) {
        const uint8_t* p = img.ptr<uint8_t>((int)r);
        out.insert(out.end(), p, p + rowb);  // little-endian host samples
    }
    std::ofstream f(path, std::ios::binary);
    if (!f.write(reinterpret_cast<const char*>(out.data()), (std::streamsize)out.size()))
        throw std::runtime_error("cannot write " + path);
}

std::array<uint8_t, 3> colormap_rgb(Colormap cmap, uint8_t v) {
    const double t = v / 255.0;
    double r, g, b;
    if (cmap == Colormap::Turbo) {  // A. Mikhailov's polynomial fit of Turbo (2019)
        const double t2 = t * t, t3 = t2 * t, t4 = t3 * t, t5 = t4 * t;
        r = 0.13572138 + 4.61539260 * t - 42.66032258 * t2 + 132.13108234 * t3 - 152.94239396 * t4 + 59.28637943 * t5;
        g = 0.09140261 + 2.19418839 * t + 4.84296658 * t2 - 14.18503333 * t3 + 4.27729857 * t4 + 2.82956604 * t5;
        b = 0.10667330 + 12.64194608 * t - 60.58204836 * t2 + 110.36276771 * t3 - 89.90310912 * t4 + 27.34824973 * t5;
    } else {  // polynomial fit of matplotlib's viridis
        static const double c[7][3] = {{0.2777273272234177, 0.005407344544966578, 0.3340998053353061},
                                       {0.1050930431085774, 1.404613529898575, 1.384590162594685},
                                       {-0.3308618287255563, 0.214847559468213, 0.09509516302823659},
                                       {-4.634230498983486, -5.799100973351585, -19.33244095627987},
                                       {6.228269936347081, 14.17993336680509, 56.69055260068105},
                                       {4.776384997670288, -13.74514537774601, -65.35303263337234},
                                       {-5.435455855934631, 4.645852612178535, 26.3124352495832}};
        double a[3];
        for (int k = 0; k < 3; ++k) {
            double s = c[6][k];
            for (int i = 5; i >= 0; --i) s = c[i][k] + t * s;
            a[k] = s;
        }
        r = a[0], g = a[1], b = a[2];
    }
    auto q = [](double x) { return (uint8_t)std::lround(std::min(1.0, std::max(0.0, x)) * 255.0); };
    return {q(r), q(g), q(b)};
}

std::vector<uint8_t> colorize(const BICOS::Image& img, Colormap cmap) {
    const int rows = img.rows(), cols = img.cols();
    double lo = DBL_MAX, hi = -DBL_MAX;
    for (int r = 0; r < rows; ++r)
        for (int c = 0; c < cols; ++c) {
            const double v = pixel(img, r, c);
            if (valid(img, v)) lo = std::min(lo, v), hi = std::max(hi, v);
        }
    // cv::normalize(NORM_MINMAX, 0..255, CV_8U, mask): scale 0 for a flat image
    const double scale = hi - lo > DBL_EPSILON ? 255.0 / (hi - lo) : 0.0, shift = -lo * scale;
    std::vector<uint8_t> rgb((size_t)rows * cols * 3, 0);
    for (int r = 0; r < rows; ++r)
        for (int c = 0; c < cols; ++c) {
            const double v = pixel(img, r, c);
            if (!valid(img, v)) continue;  // black
            const double x = std::nearbyint(v * scale + shift);  // saturate_cast: round half even
            const auto px = colormap_rgb(cmap, (uint8_t)std::min(255.0, std::max(0.0, x)));
            std::memcpy(&rgb[((size_t)r * cols + c) * 3], px.data(), 3);
        }
    return rgb;
}

std::array<double, 16> read_filestorage_matrix(const std::string& path, const std::string& name) {
    const std::vector<uint8_t> b = slurp(path);
    const std::string s(b.begin(), b.end());
    const bool xml = s.find("<opencv_storage>") != std::string::npos;
    size_t at = std::string::npos;
    if (xml) {
        at = s.find("<" + name + " ");
        if (at == std::string::npos) at = s.find("<" + name + ">");
    } else {
        for (size_t p = s.find(name + ":"); p != std::string::npos; p = s.find(name + ":", p + 1))
            if (p == 0 || s[p - 1] == '\n' || s[p - 1] == ' ') {
                at = p;
                break;
            }
    }
    if (at == std::string::npos) throw std::runtime_error(path + ": no matrix \"" + name + "\"");
    const std::vector<double> v = numbers_after(s, at, xml);
    if (v.size() != 16) throw std::runtime_error("matrix \"" + name + "\" is not 4x4");
    std::array<double, 16> q;
    std::copy(v.begin(), v.end(), q.begin());
    return q;
}

XyzStats write_xyz(const std::string& path, const BICOS::Image& disp,
                   const std::array<double, 16>& Q, bool allow_negative_z) {
    std::ofstream xyz(path);
    if (!xyz) throw std::runtime_error("cannot write " + path);
    XyzStats st;
    for (int y = 0; y < disp.rows(); ++y)
        for (int x = 0; x < disp.cols(); ++x) {
            const double d = pixel(disp, y, x);
            if (!valid(disp, d)) continue;
            double o[4];
            for (int i = 0; i < 4; ++i) o[i] = Q[4 * i] * x + Q[4 * i + 1] * y + Q[4 * i + 2] * d + Q[4 * i + 3];
            const double iw = 1.0 / o[3];
            const float X = (float)(o[0] * iw), Y = (float)(o[1] * iw), Z = (float)(o[2] * iw);
            if (!std::isfinite(X) || !std::isfinite(Y) || !std::isfinite(Z)) {
                ++st.nonfinite;
                continue;
            }
            if (!allow_negative_z && Z < 0.0f) {
                ++st.negative_z;
                continue;
            }
            xyz << X << ' ' << Y << ' ' << Z << '\n';
            ++st.written;
        }
    return st;
}

void read_stacks(const std::string& folder0, const std::optional<std::string>& folder1,
                 std::vector<Gray>& left, std::vector<Gray>& right) {
    namespace fs = std::filesystem;
    using Entry = std::pair<size_t, Gray>;
    std::vector<Entry> l, r;
    auto index_of = [](const std::string& fname, const char* msg) {
        size_t len = 0, idx = 0;
        while (len < fname.size() && std::isdigit((unsigned char)fname[len])) idx = idx * 10 + (fname[len++] - '0');
        if (len == 0) throw std::invalid_argument(msg);
        return idx;
    };
    auto files = [](const std::string& d) {
        std::vector<fs::path> v;
        for (const auto& e : fs::directory_iterator(d))
            if (e.is_regular_file()) v.push_back(e.path());
        return v;
    };
    if (folder1) {
        static const char* msg = "Expecting numbered files with names NN.png; e.g 0.png, 1.png...";
        for (const auto& p : files(folder0)) l.emplace_back(index_of(p.filename().string(), msg), read_gray(p.string(), true));
        for (const auto& p : files(*folder1)) r.emplace_back(index_of(p.filename().string(), msg), read_gray(p.string(), true));
    } else {
        static const char* msg =
            "Expecting numbered files with names NN_{left,right}.png; e.g.: 5_left.png, 10_right.png...";
        for (const auto& p : files(folder0)) {
            const std::string f = p.filename().string();
            if (f.find('_') == std::string::npos) throw std::invalid_argument(msg);
            const size_t idx = index_of(f, msg);
            (f.find("_left") != std::string::npos ? l : r).emplace_back(idx, read_gray(p.string(), false));
        }
    }
    if (l.size() != r.size())
        throw std::invalid_argument("Unequal number of images; left: " + std::to_string(l.size()) +
                                    ", right: " + std::to_string(r.size()));
    auto by_idx = [](const Entry& a, const Entry& b) { return a.first < b.first; };
    std::stable_sort(l.begin(), l.end(), by_idx);
    std::stable_sort(r.begin(), r.end(), by_idx);
    left.clear();
    right.clear();
    for (auto& e : l) left.push_back(std::move(e.second));
    for (auto& e : r) right.push_back(std::move(e.second));
}

}  // namespace bicos_cli
