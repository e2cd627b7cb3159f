// Host sanitizer harness for the CSV reader (kf_csv.cpp): its edge cases and a multi-chunk
// file (several parsing threads) under AddressSanitizer + UndefinedBehaviorSanitizer, each
// parse checked against strtod.  Host code only (no GPU).  Built and run by
// tests/test_sanitize.py:  make -C tools/sanitize
#include <cmath>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

extern "C" int kf_csv_shape(const char* path, int has_header, int64_t* rows, int* cols);
extern "C" int kf_csv_read(const char* path, int has_header, int ncols, double* out, int64_t ld, int64_t rows);

namespace kfmi {
static char g_err[512];
int set_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}
}  // namespace kfmi

static int failures = 0;
#define CHECK(c)                                                          \
    do {                                                                  \
        if (!(c)) {                                                       \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++failures;                                                   \
        }                                                                 \
    } while (0)

static std::string write_file(const char* dir, const char* name, const std::string& text) {
    std::string p = std::string(dir) + "/" + name;
    FILE* f = std::fopen(p.c_str(), "wb");
    std::fwrite(text.data(), 1, text.size(), f);
    std::fclose(f);
    return p;
}

// shape + read; returns the rc of the read (or of the shape)
static int read_all(const std::string& p, int hdr, int ncols, std::vector<double>& out, int64_t& rows) {
    int cols = 0;
    rows = 0;
    int rc = kf_csv_shape(p.c_str(), hdr, &rows, &cols);
    if (rc) return rc;
    out.assign(size_t(ncols) * size_t(rows > 0 ? rows : 1), -7.0);
    if (rows == 0) return 0;
    return kf_csv_read(p.c_str(), hdr, ncols, out.data(), rows, rows);
}

int main(int argc, char** argv) {
    const char* dir = argc > 1 ? argv[1] : "/tmp";
    std::vector<double> out;
    int64_t rows;
    // semantics
    CHECK(read_all(write_file(dir, "a.csv", "h1,h2,h3\n1,2,3\n4.5, -6 ,nan\n7,8,NaN\n"), 1, 3, out, rows) == 0);
    CHECK(rows == 3 && out[0] == 1 && out[1] == 4.5 && out[2] == 7 && out[4] == -6 && std::isnan(out[7]) &&
          std::isnan(out[8]));
    CHECK(read_all(write_file(dir, "crlf.csv", "a,b\r\n1,2\r\n3,4\r\n\r\n\n"), 1, 2, out, rows) == 0);
    CHECK(rows == 2 && out[0] == 1 && out[1] == 3 && out[2] == 2 && out[3] == 4);
    CHECK(read_all(write_file(dir, "empty.csv", ""), 1, 2, out, rows) == 0 && rows == 0);
    CHECK(read_all(write_file(dir, "hdr.csv", "a,b\n"), 1, 2, out, rows) == 0 && rows == 0);
    CHECK(read_all(write_file(dir, "nonl.csv", "a,b\n1,2"), 1, 2, out, rows) == 0 && rows == 1 && out[1] == 2);
    CHECK(read_all(write_file(dir, "bad.csv", "a,b\n1,x\n"), 1, 2, out, rows) != 0);
    CHECK(read_all(write_file(dir, "short.csv", "a,b,c\n1,2\n"), 1, 3, out, rows) != 0);
    CHECK(read_all(write_file(dir, "sign.csv", "a\n+-1\n"), 1, 1, out, rows) != 0);
    CHECK(read_all(write_file(dir, "inf.csv", "a,b\ninf,-Infinity\n"), 1, 2, out, rows) == 0 && std::isinf(out[0]) &&
          out[1] < 0 && std::isinf(out[1]));
    // a multi-chunk file (> 16 MiB: every parsing thread gets a chunk), rows of varying length
    std::string big = "t,a,b,c\n";
    std::vector<double> want;
    uint64_t s = 88172645463325252ull;
    auto rnd = [&] { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
    char buf[128];
    const int64_t nbig = 400000;
    for (int64_t r = 0; r < nbig; ++r) {
        for (int c = 0; c < 4; ++c) {
            const double v = (double(rnd() % 2000000001) - 1e9) * std::pow(10.0, double(int(rnd() % 13) - 6));
            if (c == 0) std::snprintf(buf, sizeof buf, "%.17g", v);
            else std::snprintf(buf, sizeof buf, ",%.*g", int(1 + rnd() % 17), v);
            big += buf;
        }
        big += (r % 7 == 0) ? "\r\n" : "\n";
    }
    const std::string pb = write_file(dir, "big.csv", big);
    CHECK(read_all(pb, 1, 4, out, rows) == 0 && rows == nbig);
    // every value against strtod on the same text
    const char* p = big.c_str() + big.find('\n') + 1;
    int64_t bad = 0;
    for (int64_t r = 0; r < nbig && r < rows; ++r) {
        for (int c = 0; c < 4; ++c) {
            char* end;
            const double v = std::strtod(p, &end);
            if (std::memcmp(&v, &out[size_t(c) * size_t(rows) + size_t(r)], 8) != 0) ++bad;
            p = end + 1;
        }
        if (p[-1] == '\r') ++p;
    }
    CHECK(bad == 0);
    // decimal -> double edge shapes, one value per row, against strtod: every significant-digit
    // count 1..21, exponents across the whole range (subnormals, overflow), halfway cases
    std::string hard = "v\n";
    std::vector<std::string> vals = {"9007199254740993", "9007199254740995", "2.2250738585072011e-308",
                                     "2.2250738585072012e-308", "4.9406564584124654e-324", "2.4703282292062327e-324",
                                     "2.4703282292062328e-324", "1.7976931348623157e308", "1.7976931348623159e308",
                                     "1e400", "1e-400", "0.1", "0.30000000000000004", "123456789012345678901",
                                     "0.000000000000000000000000000000000001", "1.", ".5", "0", "00.00e5",
                                     "7.038531e-26", "1448997445238699", "9223372036854775808",
                                     "1.00000000000000011102230246251565404236316680908203125",
                                     "8.98846567431158e307", "5e-324", "3e-324", "-0.0", "+1.5E+3"};
    const int nhard = argc > 2 ? std::atoi(argv[2]) : 300000;
    for (int i = 0; i < nhard; ++i) {
        const int nd = 1 + int(rnd() % 21);
        std::string m;
        for (int k = 0; k < nd; ++k) m += char('0' + (k == 0 ? 1 + rnd() % 9 : rnd() % 10));
        const int dot = int(rnd() % (nd + 1));
        if (dot < nd) m.insert(m.begin() + dot, '.');
        const int e = int(rnd() % 680) - 360;
        m += "e" + std::to_string(e);
        vals.push_back(m);
    }
    for (auto& x : vals) hard += x + "\n";
    const std::string ph = write_file(dir, "hard.csv", hard);
    CHECK(read_all(ph, 1, 1, out, rows) == 0 && rows == int64_t(vals.size()));
    int64_t bad2 = 0;
    for (size_t i = 0; i < vals.size() && int64_t(i) < rows; ++i) {
        const double w = std::strtod(vals[i].c_str(), nullptr);
        if (std::memcmp(&w, &out[i], 8) != 0) {
            if (bad2 < 5) std::fprintf(stderr, "mismatch %s: %.17g vs strtod %.17g\n", vals[i].c_str(), out[i], w);
            ++bad2;
        }
    }
    CHECK(bad2 == 0);
    std::printf("csv_asan: %d failure(s), %lld + %zu values checked\n", failures, (long long)nbig * 4, vals.size());
    return failures ? 1 : 0;
}
