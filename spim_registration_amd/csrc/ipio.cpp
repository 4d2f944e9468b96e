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
// (:75-82).  Double.toString, in two selectable forms (spim_set_java_version):
//   JDK 8 (default: Fiji runs Java 8): sun.misc.FloatingDecimal's digit loop
//     (BinaryToASCIIBuffer.dtoa / getChars), restated below -- a symmetric half-ulp
//     stopping test, so some values print longer than the shortest round trip
//     (2.0E23 -> "1.9999999999999998E23", 8.41E21 -> "8.409999999999999E21");
//   JDK 19+: the shortest decimal that round-trips (java_double_to_string_shortest).
// Both: plain notation for 1e-3 <= |d| < 1e7 ("12.0", "0.0015"), computerized
// scientific otherwise ("1.0E-4", "1.2345E7").
#include <cctype>
#include <cerrno>
#include <climits>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <sys/stat.h>
#include <type_traits>
#include <vector>

#include "common.hpp"

namespace spimdecon {

std::string java_double_to_string_shortest(double d) {
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


// ------------------------------------------------------------------------------ JDK 8
namespace {

// little-endian base-2^32 natural numbers, just what the digit loop needs
struct Big {
    std::vector<uint32_t> w;
    static Big of(uint64_t v) {
        Big b;
        while (v) {
            b.w.push_back(uint32_t(v));
            v >>= 32;
        }
        return b;
    }
    void trim() {
        while (!w.empty() && w.back() == 0) w.pop_back();
    }
    void mul_small(uint32_t m) {
        uint64_t c = 0;
        for (auto& x : w) {
            const uint64_t t = uint64_t(x) * m + c;
            x = uint32_t(t);
            c = t >> 32;
        }
        if (c) w.push_back(uint32_t(c));
    }
    void shl(int n) {
        if (w.empty() || n == 0) return;
        const int q = n / 32, r = n % 32;
        if (r) {
            uint32_t c = 0;
            for (auto& x : w) {
                const uint32_t nx = (x << r) | c;
                c = x >> (32 - r);
                x = nx;
            }
            if (c) w.push_back(c);
        }
        w.insert(w.begin(), size_t(q), 0u);
    }
    static int cmp(const Big& a, const Big& b) {
        if (a.w.size() != b.w.size()) return a.w.size() < b.w.size() ? -1 : 1;
        for (size_t i = a.w.size(); i-- > 0;)
            if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
        return 0;
    }
    static Big add(const Big& a, const Big& b) {
        Big r;
        const size_t n = std::max(a.w.size(), b.w.size());
        r.w.resize(n);
        uint64_t c = 0;
        for (size_t i = 0; i < n; ++i) {
            const uint64_t t = uint64_t(i < a.w.size() ? a.w[i] : 0) + (i < b.w.size() ? b.w[i] : 0) + c;
            r.w[i] = uint32_t(t);
            c = t >> 32;
        }
        if (c) r.w.push_back(uint32_t(c));
        return r;
    }
    void sub(const Big& b) {  // *this >= b
        int64_t c = 0;
        for (size_t i = 0; i < w.size(); ++i) {
            int64_t t = int64_t(w[i]) - (i < b.w.size() ? b.w[i] : 0) + c;
            c = t < 0 ? -1 : 0;
            w[i] = uint32_t(t + (t < 0 ? (int64_t(1) << 32) : 0));
        }
        trim();
    }
    static Big pow52(int p5, int p2, uint64_t mul = 1) {  // mul * 5^p5 * 2^p2
        Big b = of(mul);
        for (int i = 0; i < p5; ++i) b.mul_small(5);
        b.shl(p2);
        return b;
    }
};

constexpr int kExpShift = 52;
constexpr int kN5Bits[] = {0, 3, 5, 7, 10, 12, 14, 17, 19, 21, 24, 26, 28, 31, 33, 35, 38, 40, 42, 45, 47, 49, 52, 54, 56, 59, 61};
constexpr int kInsignificant[] = {0, 0, 0, 0, 1, 1, 1, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 5, 6, 6, 6, 6, 7, 7,
                                  7, 8, 8, 8, 9, 9, 9, 9, 10, 10, 10, 11, 11, 11, 12, 12, 12, 12, 13, 13, 13, 14,
                                  14, 14, 15, 15, 15, 15, 16, 16, 16, 17, 17, 17, 18, 18, 18, 19};

uint64_t pow5u(int n) {
    uint64_t r = 1;
    for (int i = 0; i < n; ++i) r *= 5;
    return r;
}

// FloatingDecimal.estimateDecExp: floor of a linear log10 estimate
int estimate_dec_exp(uint64_t fract_bits, int bin_exp) {
    const uint64_t b2 = (uint64_t(0x3FF) << 52) | (fract_bits & ((uint64_t(1) << 52) - 1));
    double d2;
    std::memcpy(&d2, &b2, 8);
    const double d = (d2 - 1.5) * 0.289529654 + 0.176091259 + double(bin_exp) * 0.301029995663981;
    return int(std::floor(d));
}

struct Digits {
    std::string s;   // '0'..'9'
    int dec_exponent = 0;
};

void roundup(Digits& g) {
    int i = int(g.s.size()) - 1;
    char q = g.s[i];
    if (q == '9') {
        while (q == '9' && i > 0) {
            g.s[i] = '0';
            q = g.s[--i];
        }
        if (q == '9') {  // carry out: high-order 1, the rest 0s (same digit count)
            g.dec_exponent += 1;
            g.s[0] = '1';
            return;
        }
    }
    g.s[i] = char(q + 1);
}

// one step of the int (W = 32) / long (W = 64) branches, in Java's wrapping arithmetic
template <typename J>
Digits dtoa_small(uint64_t fract_bits, int B5, int B2, int S5, int S2, int M5, int M2, int dec_exp) {
    using U = typename std::make_unsigned<J>::type;
    auto wr = [](U v) { return J(v); };
    J b = wr(U(U(fract_bits) * U(pow5u(B5))) << B2);
    const J s = wr(U(pow5u(S5)) << S2);
    J m = wr(U(pow5u(M5)) << M2);
    const J tens = wr(U(s) * U(10));
    Digits g;
    int q = int(b / s);
    b = wr(U(10) * U(b % s));
    m = wr(U(m) * U(10));
    bool low = b < m;
    bool high = wr(U(b) + U(m)) > tens;
    if (q == 0 && !high) --dec_exp;
    else g.s += char('0' + q);
    if (dec_exp < -3 || dec_exp >= 8) high = low = false;  // at least 2 digits in E-form
    while (!low && !high) {
        q = int(b / s);
        b = wr(U(10) * U(b % s));
        m = wr(U(m) * U(10));
        if (m > 0) {
            low = b < m;
            high = wr(U(b) + U(m)) > tens;
        } else {  // m overflowed
            low = high = true;
        }
        g.s += char('0' + q);
    }
    const J ldd = wr(U(U(b) << 1) - U(tens));
    g.dec_exponent = dec_exp + 1;
    if (high) {
        if (low) {
            if (ldd == 0) {
                if ((g.s.back() - '0') & 1) roundup(g);
            } else if (ldd > 0) {
                roundup(g);
            }
        } else {
            roundup(g);
        }
    }
    return g;
}

// BinaryToASCIIBuffer.dtoa (isCompatibleFormat = true)
Digits dtoa_jdk8(int bin_exp, uint64_t fract_bits, int n_sig_bits) {
    const int tail_zeros = __builtin_ctzll(fract_bits);
    const int n_fract_bits = kExpShift + 1 - tail_zeros;
    const int n_tiny_bits = std::max(0, n_fract_bits - bin_exp - 1);
    if (bin_exp <= 62 && bin_exp >= -(63 / 3) && n_tiny_bits == 0 && n_fract_bits + kN5Bits[0] < 64) {
        // an integer: its decimal digits, rounded past the significant ones
        int insignificant = 0;
        if (bin_exp > n_sig_bits) {
            const int p2 = bin_exp - n_sig_bits - 1;
            insignificant = (p2 > 1 && p2 < int(sizeof(kInsignificant) / sizeof(int))) ? kInsignificant[p2] : 0;
        }
        uint64_t lv = bin_exp >= kExpShift ? fract_bits << (bin_exp - kExpShift) : fract_bits >> (kExpShift - bin_exp);
        int dexp = 0;
        if (insignificant) {
            uint64_t p10 = 1;
            for (int i = 0; i < insignificant; ++i) p10 *= 10;
            const uint64_t res = lv % p10;
            lv /= p10;
            dexp += insignificant;
            if (res >= (p10 >> 1)) ++lv;
        }
        std::string s = std::to_string(lv);
        Digits g;
        dexp += int(s.size()) - 1;
        while (s.size() > 1 && s.back() == '0') s.pop_back();
        g.s = s;
        g.dec_exponent = dexp + 1;
        return g;
    }
    int dec_exp = estimate_dec_exp(fract_bits, bin_exp);
    const int B5 = std::max(0, -dec_exp);
    int B2 = B5 + n_tiny_bits + bin_exp;
    const int S5 = std::max(0, dec_exp);
    int S2 = S5 + n_tiny_bits;
    const int M5 = B5;
    int M2 = B2 - n_sig_bits;
    fract_bits >>= tail_zeros;
    B2 -= n_fract_bits - 1;
    const int common = std::min(B2, S2);
    B2 -= common;
    S2 -= common;
    M2 -= common;
    if (n_fract_bits == 1) M2 -= 1;  // exact powers of two
    if (M2 < 0) {
        B2 -= M2;
        S2 -= M2;
        M2 = 0;
    }
    const int bbits = n_fract_bits + B2 + (B5 < 27 ? kN5Bits[B5] : B5 * 3);
    const int tens_bits = S2 + 1 + (S5 + 1 < 27 ? kN5Bits[S5 + 1] : (S5 + 1) * 3);
    if (bbits < 64 && tens_bits < 64) {
        if (bbits < 32 && tens_bits < 32) return dtoa_small<int32_t>(fract_bits, B5, B2, S5, S2, M5, M2, dec_exp);
        return dtoa_small<int64_t>(fract_bits, B5, B2, S5, S2, M5, M2, dec_exp);
    }
    // FDBigInteger branch (the normalisation shift scales S, B, M, 10S alike)
    const Big S = Big::pow52(S5, S2);
    Big B = Big::pow52(B5, B2, fract_bits);
    Big M = Big::pow52(M5 + 1, M2 + 1);
    const Big tenS = Big::pow52(S5 + 1, S2 + 1);
    auto quo_rem = [&]() {  // q = B / S, B = 10 * (B % S)
        int q = 0;
        while (Big::cmp(B, S) >= 0) {
            B.sub(S);
            ++q;
        }
        B.mul_small(10);
        return q;
    };
    Digits g;
    int q = quo_rem();
    bool low = Big::cmp(B, M) < 0;
    bool high = Big::cmp(tenS, Big::add(B, M)) <= 0;
    if (q == 0 && !high) --dec_exp;
    else g.s += char('0' + q);
    if (dec_exp < -3 || dec_exp >= 8) high = low = false;
    while (!low && !high) {
        q = quo_rem();
        M.mul_small(10);
        low = Big::cmp(B, M) < 0;
        high = Big::cmp(tenS, Big::add(B, M)) <= 0;
        g.s += char('0' + q);
    }
    int ldd = 0;
    if (high && low) {
        Big b2 = B;
        b2.shl(1);
        ldd = Big::cmp(b2, tenS);
    }
    g.dec_exponent = dec_exp + 1;
    if (high) {
        if (low) {
            if (ldd == 0) {
                if ((g.s.back() - '0') & 1) roundup(g);
            } else if (ldd > 0) {
                roundup(g);
            }
        } else {
            roundup(g);
        }
    }
    return g;
}

int g_java_version = 8;

}  // namespace

std::string java_double_to_string_jdk8(double d) {
    uint64_t bits;
    std::memcpy(&bits, &d, 8);
    const bool neg = bits >> 63;
    uint64_t fract = bits & ((uint64_t(1) << 52) - 1);
    int bexp = int((bits >> 52) & 0x7FF);
    if (bexp == 0x7FF) return fract == 0 ? (neg ? "-Infinity" : "Infinity") : "NaN";
    int nsig;
    if (bexp == 0) {
        if (fract == 0) return neg ? "-0.0" : "0.0";
        const int lz = __builtin_clzll(fract);
        const int shift = lz - (63 - kExpShift);
        fract <<= shift;
        bexp = 1 - shift;
        nsig = 64 - lz;
    } else {
        fract |= uint64_t(1) << 52;
        nsig = kExpShift + 1;
    }
    bexp -= 1023;
    const Digits g = dtoa_jdk8(bexp, fract, nsig);
    const std::string& dg = g.s;
    const int nd = int(dg.size()), de = g.dec_exponent;
    std::string out = neg ? "-" : "";
    if (de > 0 && de < 8) {  // getChars
        const int cl = std::min(nd, de);
        out += dg.substr(0, size_t(cl));
        if (cl < de) out += std::string(size_t(de - cl), '0') + ".0";
        else out += "." + (cl < nd ? dg.substr(size_t(cl)) : std::string("0"));
    } else if (de <= 0 && de > -3) {
        out += "0." + std::string(size_t(-de), '0') + dg;
    } else {
        out += dg.substr(0, 1) + "." + (nd > 1 ? dg.substr(1) : std::string("0")) + "E";
        out += de <= 0 ? "-" + std::to_string(-de + 1) : std::to_string(de - 1);
    }
    return out;
}

void set_java_version(int jdk) {
    SD_CHECK(jdk == 8 || jdk == 19, SPIMDECON_ERR_ARG, "java version must be 8 or 19");
    g_java_version = jdk;
}

int java_version() { return g_java_version; }

std::string java_double_to_string(double d) {
    return g_java_version == 8 ? java_double_to_string_jdk8(d) : java_double_to_string_shortest(d);
}

namespace {

// Double.parseDouble of a trimmed field (FloatingDecimal.readJavaFormatString): optional
// sign, then "NaN", "Infinity", a decimal (digits with at most one '.', at least one
// digit, optional [eE][+-]digits) or a hex float (0x...p...), optional [fFdD] suffix.
// strtod alone would also take "inf", "nan", "infinity" and leading blanks.
bool parse_java_double(const std::string& t, double* out) {
    size_t i = 0;
    const size_t n = t.size();
    bool neg = false;
    if (i < n && (t[i] == '+' || t[i] == '-')) neg = t[i++] == '-';
    const std::string r = t.substr(i);
    if (r == "NaN") {
        *out = std::nan("");
        return true;
    }
    if (r == "Infinity") {
        *out = neg ? -INFINITY : INFINITY;
        return true;
    }
    std::string body = r;
    if (!body.empty() && std::strchr("fFdD", body.back())) body.pop_back();
    if (body.empty()) return false;
    const bool hex = body.size() > 1 && body[0] == '0' && (body[1] == 'x' || body[1] == 'X');
    if (hex) {
        if (body.find_first_of("pP") == std::string::npos) return false;
        for (size_t j = 2; j < body.size(); ++j)
            if (!std::isxdigit((unsigned char)body[j]) && !std::strchr(".pP+-", body[j])) return false;
    } else {
        size_t j = 0, digits = 0, dots = 0;
        for (; j < body.size() && (std::isdigit((unsigned char)body[j]) || body[j] == '.'); ++j) {
            if (body[j] == '.') ++dots;
            else ++digits;
        }
        if (digits == 0 || dots > 1) return false;
        if (j < body.size()) {
            if (body[j] != 'e' && body[j] != 'E') return false;
            ++j;
            if (j < body.size() && (body[j] == '+' || body[j] == '-')) ++j;
            if (j >= body.size()) return false;
            for (; j < body.size(); ++j)
                if (!std::isdigit((unsigned char)body[j])) return false;
        }
    }
    char* e = nullptr;
    const std::string full = (neg ? "-" : "") + body;
    *out = std::strtod(full.c_str(), &e);
    return e == full.c_str() + full.size();
}

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
    std::string line;
    bool header = false;
    int64_t n = 0;
    auto bad = [&](const char* why) {
        std::fclose(f);
        fail(SPIMDECON_ERR_ARG, std::string("malformed interest-point line in ") + path + ": " + why);
    };
    // BufferedReader.readLine: the line without its "\n", "\r\n" or "\r"
    auto read_line = [&](std::string& out) {
        out.clear();
        int c;
        bool any = false;
        while ((c = std::fgetc(f)) != EOF) {
            any = true;
            if (c == '\n') return true;
            if (c == '\r') {
                const int c2 = std::fgetc(f);
                if (c2 != '\n' && c2 != EOF) std::ungetc(c2, f);
                return true;
            }
            out += char(c);
        }
        return any;
    };
    while (read_line(line)) {
        if (!header) {  // do {} while (!in.readLine().startsWith("id"))
            header = line.compare(0, 2, "id") == 0;
            continue;
        }
        // p = line.split("\t") (trailing empty fields dropped); p[0..3].trim();
        // Integer.parseInt / Double.parseDouble (:194-199).  Any failure is an uncaught
        // exception in the reference: an empty line, fewer than 4 fields, an empty field
        std::vector<std::string> p;
        size_t a = 0;
        for (;;) {
            const size_t t = line.find('\t', a);
            p.push_back(line.substr(a, t == std::string::npos ? std::string::npos : t - a));
            if (t == std::string::npos) break;
            a = t + 1;
        }
        while (!p.empty() && p.back().empty()) p.pop_back();
        if (p.size() < 4) bad("fewer than 4 fields");
        for (auto& fld : p) {  // String.trim(): every char <= ' ' at both ends
            size_t b0 = 0, b1 = fld.size();
            while (b0 < b1 && (unsigned char)fld[b0] <= ' ') ++b0;
            while (b1 > b0 && (unsigned char)fld[b1 - 1] <= ' ') --b1;
            fld = fld.substr(b0, b1 - b0);
        }
        long long id = 0;
        {
            const std::string& t = p[0];
            size_t i = (!t.empty() && (t[0] == '+' || t[0] == '-')) ? 1 : 0;
            if (i >= t.size()) bad("bad id");
            for (size_t j = i; j < t.size(); ++j)
                if (t[j] < '0' || t[j] > '9') bad("bad id");
            errno = 0;
            id = std::strtoll(t.c_str(), nullptr, 10);
            if (errno || id < INT32_MIN || id > INT32_MAX) bad("id out of int range");
        }
        double pos[3];
        for (int d = 0; d < 3; ++d) {
            if (!parse_java_double(p[size_t(d) + 1], &pos[d])) bad("bad coordinate");
        }
        if (n < max_out && out) {
            spim_interest_point& q = out[n];
            std::memset(&q, 0, sizeof(q));
            for (int d = 0; d < 3; ++d) q.pos[d] = pos[d];
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

int spim_set_java_version(int jdk) {
    return guarded([&] { set_java_version(jdk); });
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
