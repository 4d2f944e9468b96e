// ipio.cpp -- interest-point list text files (.ip.txt), host side of the DoG path.
//
// Restates spim/fiji/spimdata/interestpoints/InterestPointList.java (paths under
// /root/reference/src/main/java/):
//   saveInterestPoints  :66-100   header "id\tx\ty\tz", then one line per point:
//                                 id \t l[0] \t l[1] \t l[2], each double printed by
//                                 Java's Double.toString (PrintWriter.println, "\n")
//   loadInterestPoints  :178-220  skips lines until one starts with "id", then splits
//                                 every line on '\t' (Integer.parseInt / Double.parseDouble)
// The file is <base_dir>/<file>.ip.txt; the parent directory is created when missing
// (:75-82).  Double.toString: the shortest decimal that round-trips (JDK 19+ rule),
// plain notation for 1e-3 <= |d| < 1e7 ("12.0", "0.0015"), computerized scientific
// otherwise ("1.0E-4", "1.2345E7").
#include <cerrno>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <sys/stat.h>
#include <vector>

#include "common.hpp"

namespace spimdecon {

std::string java_double_to_string(double d) {
    if (std::isnan(d)) return "NaN";
    if (std::isinf(d)) return d > 0 ? "Infinity" : "-Infinity";
    if (d == 0.0) return std::signbit(d) ? "-0.0" : "0.0";
    char buf[64];
    const auto r = std::to_chars(buf, buf + sizeof(buf), d, std::chars_format::scientific);
    SD_CHECK(r.ec == std::errc(), SPIMDECON_ERR_STATE, "double formatting failed");
    *r.ptr = 0;
    // buf = [-]D[.DDD]e[+-]XX -> sign, digits, decimal exponent of the first digit
    const char* p = buf;
    std::string sign;
    if (*p == '-') {
        sign = "-";
        ++p;
    }
    std::string digits;
    for (; *p && *p != 'e'; ++p)
        if (*p != '.') digits += *p;
    const int e = std::atoi(p + 1);
    while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
    const double a = std::fabs(d);
    int ee = e;
    if (digits.size() == 1) {
        // JDK 19+ rule: with a one-digit shortest decimal, the decimals of length 1 or 2
        // that round to d compete and the closest wins (MIN_VALUE -> "4.9E-324")
        char two[32];
        std::snprintf(two, sizeof(two), "%.1e", a);  // the correctly rounded 2-digit decimal
        if (std::strtod(two, nullptr) == a) {
            const long double x = a, c2 = std::strtold(two, nullptr);
            const long double c1 = std::strtold((digits + "e" + std::to_string(e)).c_str(), nullptr);
            if (std::fabs(c2 - x) < std::fabs(c1 - x)) {
                digits = std::string(1, two[0]) + two[2];
                ee = std::atoi(std::strchr(two, 'e') + 1);
                while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
            }
        }
    }
    std::string out;
    if (a >= 1e-3 && a < 1e7) {
        if (ee >= 0) {
            std::string ip = digits.substr(0, std::min<size_t>(digits.size(), size_t(ee) + 1));
            while (ip.size() < size_t(ee) + 1) ip += '0';
            std::string fp = digits.size() > size_t(ee) + 1 ? digits.substr(size_t(ee) + 1) : "0";
            out = ip + "." + fp;
        } else {
            out = "0." + std::string(size_t(-ee - 1), '0') + digits;
        }
    } else {
        out = digits.substr(0, 1) + "." + (digits.size() > 1 ? digits.substr(1) : "0") + "E" + std::to_string(ee);
    }
    return sign + out;
}

namespace {

std::string ip_path(const char* base_dir, const char* file) {
    SD_CHECK(file && *file, SPIMDECON_ERR_ARG, "empty interest-point file name");
    std::string path = (base_dir && *base_dir) ? std::string(base_dir) + "/" + file : std::string(file);
    return path + ".ip.txt";  // InterestPointList.getInterestPointsExt()
}

void make_parents(const std::string& path) {  // dir.mkdirs() (:75-82)
    for (size_t i = 1; i < path.size(); ++i) {
        if (path[i] != '/') continue;
        const std::string d = path.substr(0, i);
        if (::mkdir(d.c_str(), 0777) != 0 && errno != EEXIST)
            fail(SPIMDECON_ERR_ARG, "cannot create directory " + d + ": " + std::strerror(errno));
    }
}

}  // namespace

void save_interest_points(const char* base_dir, const char* file, const spim_interest_point* pts,
                          const int32_t* ids, int64_t n) {
    SD_CHECK(n >= 0 && (pts || n == 0), SPIMDECON_ERR_ARG, "bad interest-point list");
    const std::string path = ip_path(base_dir, file);
    make_parents(path);
    FILE* f = std::fopen(path.c_str(), "w");
    SD_CHECK(f, SPIMDECON_ERR_ARG, "cannot write " + path + ": " + std::strerror(errno));
    std::string s = "id\tx\ty\tz\n";
    for (int64_t i = 0; i < n; ++i) {
        s += std::to_string(ids ? int64_t(ids[i]) : i);
        for (int d = 0; d < 3; ++d) s += "\t" + java_double_to_string(pts[i].pos[d]);
        s += "\n";
        if (s.size() > (1 << 20)) {
            std::fwrite(s.data(), 1, s.size(), f);
            s.clear();
        }
    }
    std::fwrite(s.data(), 1, s.size(), f);
    const bool ok = std::fclose(f) == 0;
    SD_CHECK(ok, SPIMDECON_ERR_ARG, "write error on " + path);
}

void load_interest_points(const char* base_dir, const char* file, spim_interest_point* out, int32_t* ids,
                          int64_t max_out, int64_t* nout) {
    SD_CHECK(nout, SPIMDECON_ERR_ARG, "null count");
    const std::string path = ip_path(base_dir, file);
    FILE* f = std::fopen(path.c_str(), "r");
    // an IOException: loadInterestPoints prints it and returns false (:209-214)
    SD_CHECK(f, SPIMDECON_ERR_IO, "cannot read " + path + ": " + std::strerror(errno));
    std::vector<char> line(1 << 16);
    bool header = false;
    int64_t n = 0;
    while (std::fgets(line.data(), int(line.size()), f)) {
        if (!header) {  // do {} while (!in.readLine().startsWith("id"))
            header = std::strncmp(line.data(), "id", 2) == 0;
            continue;
        }
        char* s = line.data();
        if (*s == '\n' || *s == 0) continue;
        // fields split at '\t' and trimmed, as Integer.parseInt(p[0].trim()) /
        // Double.parseDouble(p[d].trim()) (:194-199): strtol / strtod skip the leading
        // blanks, skip_blanks the trailing ones
        auto skip_blanks = [](char* q) {
            while (*q == ' ' || *q == '\r' || *q == '\f' || *q == '\v') ++q;
            return q;
        };
        char* e = nullptr;
        const long id = std::strtol(s, &e, 10);
        double pos[3];
        bool ok = e != s && *(e = skip_blanks(e)) == '\t';
        for (int d = 0; d < 3 && ok; ++d) {
            s = e + 1;
            pos[d] = std::strtod(s, &e);
            ok = e != s;
            if (ok) {
                e = skip_blanks(e);
                ok = d == 2 ? (*e == '\t' || *e == '\n' || *e == 0) : *e == '\t';
            }
        }
        if (!ok) {
            std::fclose(f);
            fail(SPIMDECON_ERR_ARG, "malformed interest-point line in " + path);
        }
        if (n < max_out && out) {
            spim_interest_point& p = out[n];
            std::memset(&p, 0, sizeof(p));
            for (int d = 0; d < 3; ++d) p.pos[d] = pos[d];
            if (ids) ids[n] = int32_t(id);
        }
        ++n;
    }
    std::fclose(f);
    SD_CHECK(header, SPIMDECON_ERR_ARG, "no 'id' header line in " + path);
    *nout = n;
}

}  // namespace spimdecon

using namespace spimdecon;

extern "C" {

int spim_save_interest_points(const char* base_dir, const char* file, const spim_interest_point* pts,
                              const int32_t* ids, int64_t n) {
    return guarded([&] { save_interest_points(base_dir, file, pts, ids, n); });
}

int spim_load_interest_points(const char* base_dir, const char* file, spim_interest_point* out, int32_t* ids,
                              int64_t max_out, int64_t* nout) {
    return guarded([&] { load_interest_points(base_dir, file, out, ids, max_out, nout); });
}

int spim_java_double_to_string(double d, char* out, int cap) {
    return guarded([&] {
        SD_CHECK(out && cap > 0, SPIMDECON_ERR_ARG, "null output");
        const std::string s = java_double_to_string(d);
        SD_CHECK(int(s.size()) < cap, SPIMDECON_ERR_ARG, "output buffer too small");
        std::memcpy(out, s.c_str(), s.size() + 1);
    });
}

// SeparableConvolutionCUDALib.convolutionCPU (CUDASeparableConvolution.java:21): declared
// by the reference's interface and never called by it.  There is no CPU path in this
// library: the image is left unchanged and the call fails loudly (the Java binding is
// `void`, so the status reaches a caller only through spimdecon_last_error).
int convolutionCPU(float* image, const float* kernelX, const float* kernelY, const float* kernelZ, int kernelRX,
                   int kernelRY, int kernelRZ, int imageW, int imageH, int imageD, int outofbounds,
                   float outofboundsvalue) {
    (void)image, (void)kernelX, (void)kernelY, (void)kernelZ, (void)kernelRX, (void)kernelRY, (void)kernelRZ;
    (void)imageW, (void)imageH, (void)imageD, (void)outofbounds, (void)outofboundsvalue;
    return guarded([&] {
        fail(SPIMDECON_ERR_DEVICE, "convolutionCPU: no CPU path in libspimdecon (use convolve_N with a GPU)");
    });
}

}  // extern "C"
