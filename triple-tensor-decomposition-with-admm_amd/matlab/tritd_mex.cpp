// tritd_mex.cpp — MATLAB MEX gateway over libtritd.so (include/tritd.h).
//
//   [A,B,C,O,errHist,E] = tritd_mex('admm', D, r, opts, A0, B0, C0)
//                         D double -> tritd_admm_f64; D single -> tritd_admm_f32
//                         (O, E single; A, B, C, errHist double: MATLAB's class
//                         rules for a single D)
//   [A,B,C,errHist] = tritd_mex('als', X, r, opts, A0, B0, C0)
//                         triple_decomp_ALS (double X) -> tritd_als_f64
//   tritd_mex('devices', idx)  HIP device ordinals (0-based) the next solves
//                         shard D over (tritd_set_devices; [] clears)
//   X  = tritd_mex('triple_product', A, B, C[, 'qi'])
//   Xn = tritd_mex('unfold', X, mode)
//   Y  = tritd_mex('soft_threshold', X, lam)
//
// Called by the drop-in wrappers in this folder (triple_decomp_ADMM.m,
// triple_decomp_ADMM_outlier.m, triple_decomp_ALS.m, triple_product.m), which shadow
// fast_robust_triple_tensor/*.m when this folder is first on the path.
// Conventions follow the only MEX in the reference tree
// (other_methods/.../proximal_operator/flsa.c:113-142): double inputs via
// mxGetPr, outputs created with mxCreate*.  Inputs are never written (MATLAB
// shares arrays copy-on-write).  Errors: every resource is released before
// mexErrMsgIdAndTxt (it longjmps; destructors would not run).
//
// Build inside MATLAB:  mex -R2018a tritd_mex.cpp -I../../include -L../tritd -ltritd
#include <cstring>
#include <string>

#include "mex.h"
#include "tritd.h"

namespace {

void print_line(const char* line, void*) { mexPrintf("%s\n", line); }

// "Reference to non-existent field 'x'." exactly as MATLAB reports it for
// triple_decomp_ADMM.m:16-20 (the error is raised before any GPU work).
bool read_opts(const mxArray* s, tritd_opts* o, std::string* err) {
    std::memset(o, 0, sizeof *o);
    if (!mxIsStruct(s)) {
        *err = "opts must be a struct";
        return false;
    }
    struct F {
        const char* name;
        uint32_t bit;
    } fields[] = {{"mu", TRITD_OPT_MU},         {"rho", TRITD_OPT_RHO},
                  {"lambda", TRITD_OPT_LAMBDA}, {"lambda2", TRITD_OPT_LAMBDA2},
                  {"maxIter", TRITD_OPT_MAXITER}, {"tol", TRITD_OPT_TOL},
                  {"disp", TRITD_OPT_DISP}};
    for (const F& f : fields) {
        const mxArray* v = mxGetField(s, 0, f.name);
        if (!v) {
            *err = std::string("Reference to non-existent field '") + f.name + "'.";
            return false;
        }
        const double x = mxGetScalar(v);
        switch (f.bit) {
            case TRITD_OPT_MU: o->mu = x; break;
            case TRITD_OPT_RHO: o->rho = x; break;
            case TRITD_OPT_LAMBDA: o->lambda = x; break;
            case TRITD_OPT_LAMBDA2: o->lambda2 = x; break;
            case TRITD_OPT_MAXITER: o->maxIter = (int32_t)x; break;
            case TRITD_OPT_TOL: o->tol = x; break;
            case TRITD_OPT_DISP: o->disp = x != 0.0; break;
        }
        o->present |= f.bit;
    }
    // opts.model (this build's own field): 'cp' (default) or 'qi'
    o->model = TRITD_MODEL_CP;
    if (const mxArray* m = mxGetField(s, 0, "model")) {
        char buf[8] = {0};
        if (!mxIsChar(m) || mxGetString(m, buf, sizeof buf) != 0) {
            *err = "opts.model must be 'cp' or 'qi'";
            return false;
        }
        const std::string v(buf);
        if (v == "qi" || v == "QI")
            o->model = TRITD_MODEL_QI;
        else if (v != "cp" && v != "CP") {
            *err = "opts.model must be 'cp' or 'qi'";
            return false;
        }
    }
    return true;
}

// [n1,n2,n3] = size(X) with MATLAB's trailing-singleton rule; > 3 dims is
// refused (the reference fails at D - O, triple_decomp_ADMM.m:33)
bool size3(const mxArray* X, int64_t d[3], std::string* err) {
    const mwSize nd = mxGetNumberOfDimensions(X);
    const mwSize* dims = mxGetDimensions(X);
    if (nd > 3) {
        *err = "D must have at most 3 dimensions";
        return false;
    }
    d[0] = d[1] = d[2] = 1;
    for (mwSize k = 0; k < nd; ++k) d[k] = (int64_t)dims[k];
    return true;
}

mxArray* make3(int64_t a, int64_t b, int64_t c, mxClassID cls = mxDOUBLE_CLASS) {
    const mwSize dims[3] = {(mwSize)a, (mwSize)b, (mwSize)c};
    return mxCreateNumericArray(3, dims, cls, mxREAL);
}

// mexAtExit: the cached RCCL communicators go with the MEX (§8b Ownership)
void at_exit() { tritd_shutdown(); }
bool g_at_exit_set = false;

[[noreturn]] void fail(const char* id, const std::string& msg) {
    mexErrMsgIdAndTxt(id, "%s", msg.c_str());
    throw 0;  // not reached (mexErrMsgIdAndTxt does not return)
}

void need_double(const mxArray* a, const char* what) {
    if (!mxIsDouble(a) || mxIsComplex(a)) fail("tritd:class", std::string(what) + " must be real double");
}

// TRITD_FLAG_PINV_TOL of the solve that just returned: a MATLAB warning (the
// outputs are still returned)
void warn_flags() {
    if (tritd_last_flags() & TRITD_FLAG_PINV_TOL)
        mexWarnMsgIdAndTxt("tritd:pinvTolerance",
                           "a Gram's smallest pivot came within 1e3x of pinv's tolerance; pinv "
                           "could have truncated there (results may differ from the reference "
                           "beyond rounding)");
}

std::string status_msg(tritd_status s) {
    return std::string("libtritd: ") + tritd_last_error() + " (status " + std::to_string((int)s) + ")";
}

void do_admm(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs != 7) fail("tritd:nargin", "usage: tritd_mex('admm', D, r, opts, A0, B0, C0)");
    const mxArray* D = prhs[1];
    const bool single = mxIsSingle(D) && !mxIsComplex(D);
    if (!single) need_double(D, "D");
    int64_t n[3];
    std::string err;
    if (!size3(D, n, &err)) fail("tritd:dims", err);
    const int32_t r = (int32_t)mxGetScalar(prhs[2]);
    tritd_opts o;
    if (!read_opts(prhs[3], &o, &err))
        fail(err.rfind("Reference", 0) == 0 ? "MATLAB:nonExistentField" : "tritd:opts", err);
    for (int k = 4; k < 7; ++k) need_double(prhs[k], "initial factor");
    const int64_t R = (int64_t)r * r;
    if ((int64_t)mxGetNumberOfElements(prhs[4]) != n[0] * R ||
        (int64_t)mxGetNumberOfElements(prhs[5]) != R * n[1] ||
        (int64_t)mxGetNumberOfElements(prhs[6]) != R * n[2])
        fail("tritd:dims", "A0, B0, C0 must be n1 x r x r, r x n2 x r, r x r x n3");

    mxArray* A = make3(n[0], r, r);
    mxArray* B = make3(r, n[1], r);
    mxArray* C = make3(r, r, n[2]);
    const mxClassID cls = single ? mxSINGLE_CLASS : mxDOUBLE_CLASS;
    // O and E only when asked for: each is a full tensor to bring back over PCIe
    // (the drivers take [A,B,C,O,errHist]; E is this build's 6th output)
    mxArray* O = nlhs > 3 ? make3(n[0], n[1], n[2], cls) : nullptr;
    mxArray* E = nlhs > 5 ? make3(n[0], n[1], n[2], cls) : nullptr;
    mxArray* eh = mxCreateDoubleMatrix(o.maxIter > 0 ? o.maxIter : 0, 1, mxREAL);
    auto data = [](mxArray* x) { return x ? mxGetData(x) : nullptr; };
    int32_t k = 0;
    tritd_set_print_callback(print_line, nullptr);
    double* ehp = o.maxIter > 0 ? mxGetPr(eh) : nullptr;
    const tritd_status st =
        single ? tritd_admm_f32(static_cast<const float*>(mxGetData(D)), n[0], n[1], n[2], r, &o,
                                mxGetPr(prhs[4]), mxGetPr(prhs[5]), mxGetPr(prhs[6]), mxGetPr(A),
                                mxGetPr(B), mxGetPr(C), static_cast<float*>(data(O)),
                                static_cast<float*>(data(E)), ehp, &k, -1)
               : tritd_admm_f64(mxGetPr(D), n[0], n[1], n[2], r, &o, mxGetPr(prhs[4]),
                                mxGetPr(prhs[5]), mxGetPr(prhs[6]), mxGetPr(A), mxGetPr(B),
                                mxGetPr(C), static_cast<double*>(data(O)),
                                static_cast<double*>(data(E)), ehp, &k, -1);
    if (st != TRITD_OK) {
        for (mxArray* x : {A, B, C, O, E, eh})
            if (x) mxDestroyArray(x);
        fail(st == TRITD_ERR_OPTS ? "MATLAB:nonExistentField" : "tritd:solver", status_msg(st));
    }
    warn_flags();
    mxSetM(eh, (mwSize)k);  // errHist = errHist(1:k)  (triple_decomp_ADMM.m:68)
    mxArray* outs[6] = {A, B, C, O, eh, E};
    for (int q = 0; q < 6; ++q) {
        if (q < (nlhs > 0 ? nlhs : 1))
            plhs[q] = outs[q];
        else if (outs[q])
            mxDestroyArray(outs[q]);
    }
}

// triple_decomp_ALS.m:2-3 reads opts.maxIter, then opts.tol (nothing else)
bool read_als_opts(const mxArray* s, tritd_opts* o, std::string* err) {
    std::memset(o, 0, sizeof *o);
    if (!mxIsStruct(s)) {
        *err = "opts must be a struct";
        return false;
    }
    const mxArray* mi = mxGetField(s, 0, "maxIter");
    if (!mi) {
        *err = "Reference to non-existent field 'maxIter'.";
        return false;
    }
    const mxArray* tl = mxGetField(s, 0, "tol");
    if (!tl) {
        *err = "Reference to non-existent field 'tol'.";
        return false;
    }
    o->maxIter = (int32_t)mxGetScalar(mi);
    o->tol = mxGetScalar(tl);
    o->present = TRITD_OPT_MAXITER | TRITD_OPT_TOL;
    return true;
}

void do_als(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs != 7) fail("tritd:nargin", "usage: tritd_mex('als', X, r, opts, A0, B0, C0)");
    need_double(prhs[1], "X");
    int64_t n[3];
    std::string err;
    if (!size3(prhs[1], n, &err)) fail("tritd:dims", err);
    const int32_t r = (int32_t)mxGetScalar(prhs[2]);
    tritd_opts o;
    if (!read_als_opts(prhs[3], &o, &err)) fail("MATLAB:nonExistentField", err);
    for (int k = 4; k < 7; ++k) need_double(prhs[k], "initial factor");
    const int64_t R = (int64_t)r * r;
    if ((int64_t)mxGetNumberOfElements(prhs[4]) != n[0] * R ||
        (int64_t)mxGetNumberOfElements(prhs[5]) != R * n[1] ||
        (int64_t)mxGetNumberOfElements(prhs[6]) != R * n[2])
        fail("tritd:dims", "A0, B0, C0 must be n1 x r x r, r x n2 x r, r x r x n3");
    mxArray* A = make3(n[0], r, r);
    mxArray* B = make3(r, n[1], r);
    mxArray* C = make3(r, r, n[2]);
    mxArray* eh = mxCreateDoubleMatrix(o.maxIter > 0 ? o.maxIter : 0, 1, mxREAL);
    int32_t k = 0;
    tritd_set_print_callback(print_line, nullptr);
    const tritd_status st = tritd_als_f64(mxGetPr(prhs[1]), n[0], n[1], n[2], r, &o,
                                          mxGetPr(prhs[4]), mxGetPr(prhs[5]), mxGetPr(prhs[6]),
                                          mxGetPr(A), mxGetPr(B), mxGetPr(C),
                                          o.maxIter > 0 ? mxGetPr(eh) : nullptr, &k, -1);
    if (st != TRITD_OK) {
        for (mxArray* x : {A, B, C, eh}) mxDestroyArray(x);
        fail(st == TRITD_ERR_OPTS ? "MATLAB:nonExistentField" : "tritd:solver", status_msg(st));
    }
    warn_flags();
    mxSetM(eh, (mwSize)k);  // errHist = errHist(1:k)  (triple_decomp_ALS.m:21)
    mxArray* outs[4] = {A, B, C, eh};
    for (int q = 0; q < 4; ++q) {
        if (q < (nlhs > 0 ? nlhs : 1))
            plhs[q] = outs[q];
        else
            mxDestroyArray(outs[q]);
    }
}

// [A,B,C,O,errHist] = tritd_mex('ncvx', X, r, rho, lambda, gamma_A, epsilon, p, theta,
//                                maxIter, tol, A0, B0, C0)   (fast_robust_triple_tensor/test.m:1)
void do_ncvx(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs != 14)
        fail("tritd:nargin", "usage: tritd_mex('ncvx', X, r, rho, lambda, gamma_A, epsilon, p, "
                             "theta, maxIter, tol, A0, B0, C0)");
    need_double(prhs[1], "X");
    int64_t n[3];
    std::string err;
    if (!size3(prhs[1], n, &err)) fail("tritd:dims", err);
    const int32_t r = (int32_t)mxGetScalar(prhs[2]);
    double prm[6];
    for (int q = 0; q < 6; ++q) prm[q] = mxGetScalar(prhs[3 + q]);
    const int32_t maxIter = (int32_t)mxGetScalar(prhs[9]);
    const double tol = mxGetScalar(prhs[10]);
    for (int k = 11; k < 14; ++k) need_double(prhs[k], "initial factor");
    const int64_t R = (int64_t)r * r;
    if ((int64_t)mxGetNumberOfElements(prhs[11]) != n[0] * R ||
        (int64_t)mxGetNumberOfElements(prhs[12]) != R * n[1] ||
        (int64_t)mxGetNumberOfElements(prhs[13]) != R * n[2])
        fail("tritd:dims", "A0, B0, C0 must be n1 x r x r, r x n2 x r, r x r x n3");
    mxArray* A = make3(n[0], r, r);
    mxArray* B = make3(r, n[1], r);
    mxArray* C = make3(r, r, n[2]);
    mxArray* O = make3(n[0], n[1], n[2]);
    mxArray* eh = mxCreateDoubleMatrix(maxIter > 0 ? maxIter : 0, 1, mxREAL);
    int32_t k = 0;
    tritd_set_print_callback(print_line, nullptr);
    const tritd_status st = tritd_ncvx_f64(
        mxGetPr(prhs[1]), n[0], n[1], n[2], r, prm[0], prm[1], prm[2], prm[3], prm[4], prm[5],
        maxIter, tol, mxGetPr(prhs[11]), mxGetPr(prhs[12]), mxGetPr(prhs[13]), mxGetPr(A),
        mxGetPr(B), mxGetPr(C), mxGetPr(O), maxIter > 0 ? mxGetPr(eh) : nullptr, &k, -1);
    if (st != TRITD_OK) {
        for (mxArray* x : {A, B, C, O, eh}) mxDestroyArray(x);
        fail("tritd:solver", status_msg(st));
    }
    warn_flags();
    mxSetM(eh, (mwSize)k);  // errHist(1:k) on a break (test.m:66); maxIter entries otherwise
    mxArray* outs[5] = {A, B, C, O, eh};
    for (int q = 0; q < 5; ++q) {
        if (q < (nlhs > 0 ? nlhs : 1))
            plhs[q] = outs[q];
        else
            mxDestroyArray(outs[q]);
    }
}

void do_devices(int, mxArray*[], int nrhs, const mxArray* prhs[]) {
    if (nrhs != 2) fail("tritd:nargin", "usage: tritd_mex('devices', idx)");
    need_double(prhs[1], "idx");
    const size_t n = mxGetNumberOfElements(prhs[1]);
    if (n > 16) fail("tritd:devices", "at most 16 devices");
    int32_t d[16];
    const double* v = mxGetPr(prhs[1]);
    for (size_t q = 0; q < n; ++q) {
        if (v[q] != (double)(int32_t)v[q]) fail("tritd:devices", "device ordinals must be integers");
        d[q] = (int32_t)v[q];
    }
    const tritd_status st = tritd_set_devices(d, (int32_t)n);
    if (st != TRITD_OK) fail("tritd:devices", status_msg(st));
}

void do_triple_product(int, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs != 4 && nrhs != 5)
        fail("tritd:nargin", "usage: tritd_mex('triple_product', A, B, C[, 'qi'])");
    bool qi = false;
    if (nrhs == 5) {
        char buf[8] = {0};
        if (!mxIsChar(prhs[4]) || mxGetString(prhs[4], buf, sizeof buf) != 0 ||
            (std::string(buf) != "qi" && std::string(buf) != "cp"))
            fail("tritd:model", "model must be 'cp' or 'qi'");
        qi = std::string(buf) == "qi";
    }
    for (int k = 1; k < 4; ++k) need_double(prhs[k], "factor");
    int64_t a[3], b[3], c[3];
    std::string err;
    if (!size3(prhs[1], a, &err) || !size3(prhs[2], b, &err) || !size3(prhs[3], c, &err))
        fail("tritd:dims", err);
    mxArray* X = make3(a[0], b[1], c[2]);
    const tritd_status st =
        (qi ? tritd_triple_product_qi_f64 : tritd_triple_product_f64)(
            mxGetPr(prhs[1]), mxGetPr(prhs[2]), mxGetPr(prhs[3]), a[0], b[1], c[2], (int32_t)a[1],
            mxGetPr(X));
    if (st != TRITD_OK) {
        mxDestroyArray(X);
        fail("tritd:triple_product", status_msg(st));
    }
    plhs[0] = X;
}

void do_unfold(int, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs != 3) fail("tritd:nargin", "usage: tritd_mex('unfold', X, mode)");
    need_double(prhs[1], "X");
    int64_t n[3];
    std::string err;
    if (!size3(prhs[1], n, &err)) fail("tritd:dims", err);
    const int mode = (int)mxGetScalar(prhs[2]);
    if (mode < 1 || mode > 3) fail("tritd:unfold", "Mode must be 1, 2, or 3.");  // unfold.m:12
    const int64_t rows = mode == 1 ? n[0] : (mode == 2 ? n[1] : n[2]);
    mxArray* Xn = mxCreateDoubleMatrix((mwSize)rows, (mwSize)(n[0] * n[1] * n[2] / rows), mxREAL);
    const tritd_status st = tritd_unfold_f64(mxGetPr(prhs[1]), n[0], n[1], n[2], mode, mxGetPr(Xn));
    if (st != TRITD_OK) {
        mxDestroyArray(Xn);
        fail("tritd:unfold", status_msg(st));
    }
    plhs[0] = Xn;
}

void do_soft_threshold(int, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs != 3) fail("tritd:nargin", "usage: tritd_mex('soft_threshold', X, lam)");
    need_double(prhs[1], "X");
    mxArray* Y = mxCreateNumericArray(mxGetNumberOfDimensions(prhs[1]), mxGetDimensions(prhs[1]),
                                      mxDOUBLE_CLASS, mxREAL);
    const tritd_status st = tritd_soft_threshold_f64(mxGetPr(prhs[1]),
                                                     (int64_t)mxGetNumberOfElements(prhs[1]),
                                                     mxGetScalar(prhs[2]), mxGetPr(Y));
    if (st != TRITD_OK) {
        mxDestroyArray(Y);
        fail("tritd:soft_threshold", status_msg(st));
    }
    plhs[0] = Y;
}

}  // namespace

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs < 1 || !mxIsChar(prhs[0])) fail("tritd:nargin", "first argument must be a command string");
    char cmd[32] = {0};
    mxGetString(prhs[0], cmd, sizeof cmd);
    const std::string c(cmd);
    if (!g_at_exit_set) {
        mexAtExit(at_exit);
        g_at_exit_set = true;
    }
    if (c == "devices")
        do_devices(nlhs, plhs, nrhs, prhs);
    else if (c == "admm")
        do_admm(nlhs, plhs, nrhs, prhs);
    else if (c == "als")
        do_als(nlhs, plhs, nrhs, prhs);
    else if (c == "ncvx")
        do_ncvx(nlhs, plhs, nrhs, prhs);
    else if (c == "triple_product")
        do_triple_product(nlhs, plhs, nrhs, prhs);
    else if (c == "unfold")
        do_unfold(nlhs, plhs, nrhs, prhs);
    else if (c == "soft_threshold")
        do_soft_threshold(nlhs, plhs, nrhs, prhs);
    else
        fail("tritd:cmd", "unknown command '" + c + "'");
}
