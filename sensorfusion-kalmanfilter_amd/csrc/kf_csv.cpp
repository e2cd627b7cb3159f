// Native numeric CSV reader for the ingest path (kf_csv_shape / kf_csv_read, include/kf.h).
//
// Replaces KF_SensorFusion.load_data_from_csv (kf_workers.py:290-298), which keeps every field
// as a Python string and converts it with float() at each use (kf_workers.py:313-316, 339-340,
// 353-357, 380-383).  Here the file is memory-mapped, split into newline-aligned chunks parsed
// by one thread each, and every requested column lands in a column-major double array, ready
// for one host->device copy.  Conversion semantics match the reference's:
//   * a field containing "nan" in any case (the reference's `'nan' in s.lower()` test,
//     kf_workers.py:310, 336) becomes a quiet NaN;
//   * otherwise the field is parsed as Python's float() does (correctly rounded, surrounding
//     blanks ignored, optional sign, "inf"/"infinity"); anything else is an error, like the
//     ValueError float() would raise.
// Quoted fields are not supported (numeric logs have none).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <charconv>
#include <cerrno>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kf.h"
#include "kf_internal.h"

namespace {

struct Mapped {
    const char* p = nullptr;
    size_t n = 0;
    int fd = -1;
    ~Mapped() {
        if (p && n) munmap(const_cast<char*>(p), n);
        if (fd >= 0) close(fd);
    }
};

int map_file(const char* path, Mapped& m) {
    if (!path) return kfmi::set_error(KF_EINVAL, "kf_csv: null path");
    m.fd = open(path, O_RDONLY);
    if (m.fd < 0) return kfmi::set_error(KF_EINVAL, "kf_csv: cannot open %s: %s", path, std::strerror(errno));
    struct stat st;
    if (fstat(m.fd, &st) != 0) return kfmi::set_error(KF_EINVAL, "kf_csv: cannot stat %s", path);
    m.n = static_cast<size_t>(st.st_size);
    if (m.n == 0) return KF_OK;
    void* p = mmap(nullptr, m.n, PROT_READ, MAP_PRIVATE, m.fd, 0);
    if (p == MAP_FAILED) {
        m.n = 0;
        return kfmi::set_error(KF_EINVAL, "kf_csv: cannot map %s", path);
    }
    madvise(p, m.n, MADV_SEQUENTIAL);
    m.p = static_cast<const char*>(p);
    return KF_OK;
}

// [begin, end) of the data rows (header skipped).
void data_range(const Mapped& m, int has_header, const char*& b, const char*& e) {
    b = m.p;
    e = m.p + m.n;
    if (has_header && b < e) {
        const char* nl = static_cast<const char*>(std::memchr(b, '\n', e - b));
        b = nl ? nl + 1 : e;
    }
}

// A line is [s, t) without its '\n'; a trailing '\r' is dropped by the field parser.
inline bool blank_line(const char* s, const char* t) {
    for (; s < t; ++s)
        if (*s != '\r' && *s != ' ' && *s != '\t') return false;
    return true;
}

int64_t count_rows(const char* b, const char* e) {
    int64_t n = 0;
    const char* s = b;
    while (s < e) {
        const char* nl = static_cast<const char*>(std::memchr(s, '\n', e - s));
        ++n;
        s = nl ? nl + 1 : e;
    }
    return n;
}

inline bool has_nan_text(const char* s, const char* t) {
    for (; s + 3 <= t; ++s)
        if ((s[0] | 0x20) == 'n' && (s[1] | 0x20) == 'a' && (s[2] | 0x20) == 'n') return true;
    return false;
}

// float() semantics on [s, t); returns false on a malformed field.
inline bool parse_field(const char* s, const char* t, double& v) {
    while (s < t && (*s == ' ' || *s == '\t')) ++s;
    while (t > s && (t[-1] == ' ' || t[-1] == '\t' || t[-1] == '\r')) --t;
    if (s == t) return false;
    if (has_nan_text(s, t)) {
        v = std::nan("");
        return true;
    }
    bool neg = false;
    if (*s == '+' || *s == '-') {
        neg = *s == '-';
        ++s;
    }
    if (s == t || *s == '+' || *s == '-') return false;
    auto r = std::from_chars(s, t, v, std::chars_format::general);
    if (r.ec == std::errc::result_out_of_range && r.ptr == t) {
        // float() gives inf, 0.0 or a subnormal there; from_chars leaves v unset: strtod rounds
        // it (the C locale's '.', a NUL-terminated copy of the field)
        const std::string f(s, t);
        v = std::strtod(f.c_str(), nullptr);
        r.ec = std::errc();
    }
    if (r.ec != std::errc() || r.ptr != t) return false;
    if (neg) v = -v;
    return true;
}

struct Chunk {
    const char* b;
    const char* e;
    int64_t row0;
    int64_t rows;
    int err_code = KF_OK;
    int64_t err_row = -1;
    int err_col = -1;
    int err_fields = -1;
};

int n_threads(size_t bytes) {
    unsigned hw = std::thread::hardware_concurrency();
    int t = static_cast<int>(std::min<unsigned>(hw ? hw : 1, 16));
    const size_t per = size_t(1) << 20;  // no point splitting below ~1 MiB per thread
    return std::max(1, std::min<int>(t, static_cast<int>(bytes / per) + 1));
}

// newline-aligned chunks of [b, e), one per thread
std::vector<std::pair<const char*, const char*>> split_lines(const char* b, const char* e) {
    const int nt = n_threads(static_cast<size_t>(e - b));
    std::vector<std::pair<const char*, const char*>> ch;
    const char* s = b;
    for (int i = 0; i < nt && s < e; ++i) {
        const char* t = (i == nt - 1) ? e : b + (e - b) * (i + 1) / nt;
        if (t < s) t = s;
        if (t < e) {
            const char* nl = static_cast<const char*>(std::memchr(t, '\n', e - t));
            t = nl ? nl + 1 : e;
        }
        ch.emplace_back(s, t);
        s = t;
    }
    return ch;
}

// count_rows over newline-aligned chunks in parallel (a line never straddles two chunks, so the
// per-chunk counts add up)
int64_t count_rows_parallel(const char* b, const char* e) {
    const auto ch = split_lines(b, e);
    std::vector<int64_t> n(ch.size(), 0);
    std::vector<std::thread> th;
    for (size_t i = 0; i < ch.size(); ++i) th.emplace_back([&, i] { n[i] = count_rows(ch[i].first, ch[i].second); });
    for (auto& t : th) t.join();
    int64_t total = 0;
    for (int64_t v : n) total += v;
    return total;
}

}  // namespace

extern "C" {

int kf_csv_shape(const char* path, int has_header, int64_t* rows, int* cols) {
    Mapped m;
    if (int rc = map_file(path, m)) return rc;
    const char *b, *e;
    data_range(m, has_header, b, e);
    int64_t n = count_rows_parallel(b, e);
    // trailing blank lines (a file ending in "\n\n") are not rows of data
    while (n > 0) {
        const char* le = e;
        if (le > b && le[-1] == '\n') --le;
        const char* ls = le;
        while (ls > b && ls[-1] != '\n') --ls;
        if (!blank_line(ls, le)) break;
        e = ls;
        --n;
    }
    int c = 0;
    if (n > 0) {
        const char* nl = static_cast<const char*>(std::memchr(b, '\n', e - b));
        const char* t = nl ? nl : e;
        c = 1 + static_cast<int>(std::count(b, t, ','));
    }
    if (rows) *rows = n;
    if (cols) *cols = c;
    return KF_OK;
}

int kf_csv_read(const char* path, int has_header, int ncols, double* out, int64_t ld, int64_t rows) {
    if (ncols < 1 || !out) return kfmi::set_error(KF_EINVAL, "kf_csv_read: ncols = %d, out = %p", ncols, (void*)out);
    if (ld < rows || rows < 0) return kfmi::set_error(KF_EINVAL, "kf_csv_read: ld %lld < rows %lld",
                                                      (long long)ld, (long long)rows);
    Mapped m;
    if (int rc = map_file(path, m)) return rc;
    const char *b, *e;
    data_range(m, has_header, b, e);
    // newline-aligned chunks, one per thread
    std::vector<Chunk> ch;
    for (const auto& c : split_lines(b, e)) ch.push_back(Chunk{c.first, c.second, 0, 0});
    {
        std::vector<std::thread> th;
        for (auto& c : ch) th.emplace_back([&c] { c.rows = count_rows(c.b, c.e); });
        for (auto& t : th) t.join();
    }
    int64_t total = 0;
    for (auto& c : ch) {
        c.row0 = total;
        total += c.rows;
    }
    auto parse = [&](Chunk& c) {
        int64_t r = c.row0;
        const char* p = c.b;
        while (p < c.e) {
            const char* nl = static_cast<const char*>(std::memchr(p, '\n', c.e - p));
            const char* t = nl ? nl : c.e;
            if (r >= rows) {
                if (!blank_line(p, t)) {
                    c.err_code = KF_EINVAL;
                    c.err_row = r;
                }
                return;
            }
            const char* f = p;
            int col = 0;
            while (col < ncols) {
                const char* comma = static_cast<const char*>(std::memchr(f, ',', t - f));
                const char* fe = comma ? comma : t;
                double v;
                if (!parse_field(f, fe, v)) {
                    c.err_code = KF_EINVAL;
                    c.err_row = r;
                    c.err_col = col;
                    c.err_fields = 1 + static_cast<int>(std::count(p, t, ','));
                    return;
                }
                out[int64_t(col) * ld + r] = v;
                ++col;
                if (!comma) break;
                f = comma + 1;
            }
            if (col < ncols) {
                c.err_code = KF_EINVAL;
                c.err_row = r;
                c.err_fields = col;
                return;
            }
            ++r;
            p = nl ? nl + 1 : c.e;
        }
    };
    {
        std::vector<std::thread> th;
        for (auto& c : ch) th.emplace_back([&parse, &c] { parse(c); });
        for (auto& t : th) t.join();
    }
    for (auto& c : ch) {
        if (c.err_code == KF_OK) continue;
        if (c.err_row >= rows)
            return kfmi::set_error(KF_EINVAL, "kf_csv_read: %s has more than %lld data rows", path, (long long)rows);
        if (c.err_col >= 0)
            return kfmi::set_error(KF_EINVAL, "kf_csv_read: %s data row %lld column %d is not a number", path,
                                   (long long)c.err_row, c.err_col);
        return kfmi::set_error(KF_EINVAL, "kf_csv_read: %s data row %lld has %d fields, expected >= %d", path,
                               (long long)c.err_row, c.err_fields, ncols);
    }
    if (total < rows)
        return kfmi::set_error(KF_EINVAL, "kf_csv_read: %s has %lld data rows, expected %lld", path,
                               (long long)total, (long long)rows);
    return KF_OK;
}

}  // extern "C"
