// Mock mx runtime + a C entry point that drives mexFunction — TEST ONLY.
#include "mex.h"

#include <cstdio>
#include <cstring>
#include <map>
#include <vector>

struct mxArray {
    mxClassID cls = mxDOUBLE_CLASS;
    std::vector<mwSize> dims;
    std::vector<double> data;  // mxDOUBLE_CLASS
    std::vector<float> fdata;  // mxSINGLE_CLASS
    std::string str;
    std::map<std::string, mxArray*> fields;
};

static std::string g_printed;

bool mxIsStruct(const mxArray* a) { return a->cls == mxSTRUCT_CLASS; }
bool mxIsDouble(const mxArray* a) { return a->cls == mxDOUBLE_CLASS; }
bool mxIsSingle(const mxArray* a) { return a->cls == mxSINGLE_CLASS; }
bool mxIsComplex(const mxArray*) { return false; }
bool mxIsChar(const mxArray* a) { return a->cls == mxCHAR_CLASS; }
mxArray* mxGetField(const mxArray* a, size_t, const char* n) {
    auto it = a->fields.find(n);
    return it == a->fields.end() ? nullptr : it->second;
}
double mxGetScalar(const mxArray* a) { return a->data.empty() ? 0.0 : a->data[0]; }
mwSize mxGetNumberOfDimensions(const mxArray* a) { return a->dims.size(); }
const mwSize* mxGetDimensions(const mxArray* a) { return a->dims.data(); }
size_t mxGetNumberOfElements(const mxArray* a) {
    size_t n = 1;
    for (auto d : a->dims) n *= d;
    return n;
}
double* mxGetPr(const mxArray* a) { return const_cast<double*>(a->data.data()); }
void* mxGetData(const mxArray* a) {
    return a->cls == mxSINGLE_CLASS ? static_cast<void*>(const_cast<float*>(a->fdata.data()))
                                    : static_cast<void*>(const_cast<double*>(a->data.data()));
}
void mxSetM(mxArray* a, mwSize m) { a->dims[0] = m; }
int mxGetString(const mxArray* a, char* buf, mwSize n) {
    std::snprintf(buf, n, "%s", a->str.c_str());
    return 0;
}
mxArray* mxCreateNumericArray(mwSize nd, const mwSize* d, mxClassID c, mxComplexity) {
    auto* a = new mxArray;
    a->cls = c;
    a->dims.assign(d, d + nd);
    if (c == mxSINGLE_CLASS)
        a->fdata.assign(mxGetNumberOfElements(a), 0.0f);
    else
        a->data.assign(mxGetNumberOfElements(a), 0.0);
    return a;
}
mxArray* mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity c) {
    const mwSize d[2] = {m, n};
    return mxCreateNumericArray(2, d, mxDOUBLE_CLASS, c);
}
void mxDestroyArray(mxArray* a) {
    for (auto& f : a->fields) mxDestroyArray(f.second);
    delete a;
}
void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    throw MockMexError{id, buf};
}
// MATLAB prints "Warning: <msg>" and returns; the mock records it with the
// printed text
void mexWarnMsgIdAndTxt(const char* id, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_printed += std::string("Warning [") + id + "]: " + buf + "\n";
}
int mexPrintf(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    const int n = std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_printed += buf;
    return n;
}

static void (*g_at_exit)(void) = nullptr;
int mexAtExit(void (*fn)(void)) {
    g_at_exit = fn;
    return 0;
}

static mxArray* sgl(const float* p, std::vector<mwSize> dims) {
    mxArray* a = mxCreateNumericArray(dims.size(), dims.data(), mxSINGLE_CLASS, mxREAL);
    if (!a->fdata.empty()) std::memcpy(a->fdata.data(), p, a->fdata.size() * sizeof(float));
    return a;
}

static mxArray* dbl(const double* p, std::vector<mwSize> dims) {
    mxArray* a = mxCreateNumericArray(dims.size(), dims.data(), mxDOUBLE_CLASS, mxREAL);
    // (an empty array may come with a null pointer: memcpy's arguments must
    // not be null even for zero bytes — UBSan, tests/test_sanitizers.py)
    if (!a->data.empty()) std::memcpy(a->data.data(), p, a->data.size() * sizeof(double));
    return a;
}

extern "C" {
static mxArray* cmd_arg(const char* c) {
    auto* cmd = new mxArray;
    cmd->cls = mxCHAR_CLASS;
    cmd->str = c;
    cmd->dims = {1, std::strlen(c)};
    return cmd;
}

// tritd_mex('devices', devs) (n = 0: an empty matrix); returns 0 or 1 + err
int mock_devices(const double* devs, int n, char* err, int errlen) {
    mxArray* in[2] = {cmd_arg("devices"), dbl(devs, {1, (mwSize)n})};
    int rc = 0;
    try {
        mexFunction(0, nullptr, 2, const_cast<const mxArray**>(in));
    } catch (const MockMexError& e) {
        std::snprintf(err, errlen, "%s|%s", e.id.c_str(), e.msg.c_str());
        rc = 1;
    }
    for (auto* a : in) mxDestroyArray(a);
    return rc;
}

// MATLAB clearing the MEX: runs the function registered with mexAtExit
int mock_clear(void) {
    if (!g_at_exit) return 1;
    g_at_exit();
    g_at_exit = nullptr;
    return 0;
}

// opt_names: comma-separated field names present in opts; opt_vals in the same order.
// single != 0: D, O, E are float (a D of class single).
int mock_admm(const void* D, long n1, long n2, long n3, int r, const char* opt_names,
              const double* opt_vals, const double* A0, const double* B0, const double* C0,
              double* A, double* B, double* C, void* O, void* E, double* errHist, int* k,
              char* err, int errlen, char* printed, int printlen, int single) {
    std::vector<mxArray*> in;
    in.push_back(cmd_arg("admm"));
    if (single)
        in.push_back(sgl(static_cast<const float*>(D), {(mwSize)n1, (mwSize)n2, (mwSize)n3}));
    else
        in.push_back(dbl(static_cast<const double*>(D), {(mwSize)n1, (mwSize)n2, (mwSize)n3}));
    double rr = r;
    in.push_back(dbl(&rr, {1, 1}));
    auto* opts = new mxArray;
    opts->cls = mxSTRUCT_CLASS;
    opts->dims = {1, 1};
    {
        std::string names(opt_names);
        size_t pos = 0;
        int q = 0;
        while (pos <= names.size() && !names.empty()) {
            const size_t c = names.find(',', pos);
            const std::string nm = names.substr(pos, c == std::string::npos ? std::string::npos : c - pos);
            const size_t eq = nm.find('=');
            if (eq != std::string::npos)  // "model=qi": a char field, no value consumed
                opts->fields[nm.substr(0, eq)] = cmd_arg(nm.substr(eq + 1).c_str());
            else
                opts->fields[nm] = dbl(&opt_vals[q++], {1, 1});
            if (c == std::string::npos) break;
            pos = c + 1;
        }
    }
    in.push_back(opts);
    in.push_back(dbl(A0, {(mwSize)n1, (mwSize)r, (mwSize)r}));
    in.push_back(dbl(B0, {(mwSize)r, (mwSize)n2, (mwSize)r}));
    in.push_back(dbl(C0, {(mwSize)r, (mwSize)r, (mwSize)n3}));
    mxArray* out[6] = {nullptr};
    int rc = 0;
    g_printed.clear();
    try {
        // E == NULL: the drivers' five-output call [A,B,C,O,errHist] (nargout 5)
        const int nlhs = E ? 6 : 5;
        mexFunction(nlhs, out, (int)in.size(), const_cast<const mxArray**>(in.data()));
        if (nlhs == 5 && out[5]) throw MockMexError{"mock:nlhs", "a 6th output for nargout 5"};
        const size_t nA = (size_t)n1 * r * r, nB = (size_t)r * n2 * r, nC = (size_t)r * r * n3;
        const size_t N = (size_t)n1 * n2 * n3;
        std::memcpy(A, out[0]->data.data(), nA * 8);
        std::memcpy(B, out[1]->data.data(), nB * 8);
        std::memcpy(C, out[2]->data.data(), nC * 8);
        const size_t es = single ? 4 : 8;
        if ((out[3]->cls == mxSINGLE_CLASS) != (single != 0) ||
            (E && (out[5]->cls == mxSINGLE_CLASS) != (single != 0)))
            throw MockMexError{"mock:class", "O/E class differs from the class of D"};
        std::memcpy(O, mxGetData(out[3]), N * es);
        *k = (int)out[4]->dims[0];
        std::memcpy(errHist, out[4]->data.data(), (size_t)*k * 8);
        if (E) std::memcpy(E, mxGetData(out[5]), N * es);
    } catch (const MockMexError& e) {
        std::snprintf(err, errlen, "%s|%s", e.id.c_str(), e.msg.c_str());
        rc = 1;
    }
    std::snprintf(printed, printlen, "%s", g_printed.c_str());
    for (auto* a : in) mxDestroyArray(a);
    for (auto* a : out)
        if (a) mxDestroyArray(a);
    return rc;
}

// [A,B,C,errHist] = tritd_mex('als', X, r, opts, A0, B0, C0)
int mock_als(const double* X, long n1, long n2, long n3, int r, const char* opt_names,
             const double* opt_vals, const double* A0, const double* B0, const double* C0,
             double* A, double* B, double* C, double* errHist, int* k, char* err, int errlen,
             char* printed, int printlen) {
    std::vector<mxArray*> in;
    in.push_back(cmd_arg("als"));
    in.push_back(dbl(X, {(mwSize)n1, (mwSize)n2, (mwSize)n3}));
    double rr = r;
    in.push_back(dbl(&rr, {1, 1}));
    auto* opts = new mxArray;
    opts->cls = mxSTRUCT_CLASS;
    opts->dims = {1, 1};
    {
        std::string names(opt_names);
        size_t pos = 0;
        int q = 0;
        while (pos <= names.size() && !names.empty()) {
            const size_t c = names.find(',', pos);
            const std::string nm = names.substr(pos, c == std::string::npos ? std::string::npos : c - pos);
            opts->fields[nm] = dbl(&opt_vals[q++], {1, 1});
            if (c == std::string::npos) break;
            pos = c + 1;
        }
    }
    in.push_back(opts);
    in.push_back(dbl(A0, {(mwSize)n1, (mwSize)r, (mwSize)r}));
    in.push_back(dbl(B0, {(mwSize)r, (mwSize)n2, (mwSize)r}));
    in.push_back(dbl(C0, {(mwSize)r, (mwSize)r, (mwSize)n3}));
    mxArray* out[4] = {nullptr};
    int rc = 0;
    g_printed.clear();
    try {
        mexFunction(4, out, (int)in.size(), const_cast<const mxArray**>(in.data()));
        std::memcpy(A, out[0]->data.data(), (size_t)n1 * r * r * 8);
        std::memcpy(B, out[1]->data.data(), (size_t)r * n2 * r * 8);
        std::memcpy(C, out[2]->data.data(), (size_t)r * r * n3 * 8);
        *k = (int)out[3]->dims[0];
        std::memcpy(errHist, out[3]->data.data(), (size_t)*k * 8);
    } catch (const MockMexError& e) {
        std::snprintf(err, errlen, "%s|%s", e.id.c_str(), e.msg.c_str());
        rc = 1;
    }
    std::snprintf(printed, printlen, "%s", g_printed.c_str());
    for (auto* a : in) mxDestroyArray(a);
    for (auto* a : out)
        if (a) mxDestroyArray(a);
    return rc;
}

// tritd_mex('ncvx', X, r, rho, lambda, gamma_A, epsilon, p, theta, maxIter, tol, A0, B0, C0)
int mock_ncvx(const double* X, long n1, long n2, long n3, int r, const double* prm8,
              const double* A0, const double* B0, const double* C0, double* A, double* B,
              double* C, double* O, double* errHist, int* k, char* err, int errlen, char* printed,
              int printlen) {
    std::vector<mxArray*> in;
    in.push_back(cmd_arg("ncvx"));
    in.push_back(dbl(X, {(mwSize)n1, (mwSize)n2, (mwSize)n3}));
    double rr = r;
    in.push_back(dbl(&rr, {1, 1}));
    for (int q = 0; q < 8; ++q) in.push_back(dbl(&prm8[q], {1, 1}));
    in.push_back(dbl(A0, {(mwSize)n1, (mwSize)r, (mwSize)r}));
    in.push_back(dbl(B0, {(mwSize)r, (mwSize)n2, (mwSize)r}));
    in.push_back(dbl(C0, {(mwSize)r, (mwSize)r, (mwSize)n3}));
    mxArray* out[5] = {nullptr};
    int rc = 0;
    g_printed.clear();
    try {
        mexFunction(5, out, (int)in.size(), const_cast<const mxArray**>(in.data()));
        std::memcpy(A, out[0]->data.data(), (size_t)n1 * r * r * 8);
        std::memcpy(B, out[1]->data.data(), (size_t)r * n2 * r * 8);
        std::memcpy(C, out[2]->data.data(), (size_t)r * r * n3 * 8);
        std::memcpy(O, out[3]->data.data(), (size_t)n1 * n2 * n3 * 8);
        *k = (int)out[4]->dims[0];
        std::memcpy(errHist, out[4]->data.data(), (size_t)*k * 8);
    } catch (const MockMexError& e) {
        std::snprintf(err, errlen, "%s|%s", e.id.c_str(), e.msg.c_str());
        rc = 1;
    }
    std::snprintf(printed, printlen, "%s", g_printed.c_str());
    for (auto* a : in) mxDestroyArray(a);
    for (auto* a : out)
        if (a) mxDestroyArray(a);
    return rc;
}
}
