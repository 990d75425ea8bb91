// TEST DOUBLE -- NOT OpenCV. OpenCV is not installed in this image, so the cv::Mat branch of
// include/BICOS/{common,match}.hpp (Image = cv::Mat, the reference's CPU build) is compiled
// against this minimal stand-in for the part of cv::Mat a BICOS caller touches: the CV_*
// type codes, Mat(rows, cols, type[, data, step]) views and owned storage, rows / cols /
// data / step[0] / type() / create() / empty() / ptr<T>() / at<T>(). Only
// tests/cpp/ref_style.cpp is built with it (tests/test_cpp_api.py); no library code is.
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <vector>

#define CV_8U 0
#define CV_16U 2
#define CV_16S 3
#define CV_32F 5
#define CV_64F 6
#define CV_8UC1 CV_8U
#define CV_16UC1 CV_16U

namespace cv {

class Mat {
public:
    struct Step {
        size_t s[2] = {0, 0};
        size_t operator[](int i) const { return s[i]; }
        operator size_t() const { return s[0]; }
    };
    int rows = 0, cols = 0;
    unsigned char* data = nullptr;
    Step step;

    Mat() = default;
    Mat(int r, int c, int type) { create(r, c, type); }
    Mat(int r, int c, int type, void* d, size_t st = 0) : rows(r), cols(c), _type(type) {
        data = static_cast<unsigned char*>(d);
        step.s[1] = esize(type);
        step.s[0] = st ? st : (size_t)c * step.s[1];
    }
    int type() const { return _type; }
    int depth() const { return _type; }
    bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
    void create(int r, int c, int type) {
        if (_buf && r == rows && c == cols && type == _type) return;
        rows = r;
        cols = c;
        _type = type;
        step.s[1] = esize(type);
        step.s[0] = (size_t)c * step.s[1];
        _buf = std::make_shared<std::vector<unsigned char>>(step.s[0] * r);
        data = _buf->data();
    }
    template <typename T>
    T* ptr(int r) const { return reinterpret_cast<T*>(data + (size_t)r * step.s[0]); }
    template <typename T>
    T& at(int r, int c) const { return ptr<T>(r)[c]; }

private:
    static size_t esize(int t) { return t == CV_8U ? 1 : t <= CV_16S ? 2 : t == CV_32F ? 4 : 8; }
    int _type = CV_8U;
    std::shared_ptr<std::vector<unsigned char>> _buf;
};

}  // namespace cv
