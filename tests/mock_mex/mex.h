// Minimal mock of the MATLAB MEX/mx API — TEST ONLY.  Lets the gateway
// (triple-tensor-decomposition-with-admm_amd/matlab/tritd_mex.cpp) be compiled
// and driven without MATLAB (no mex.h exists in this image).
// Only the calls the gateway makes are provided; semantics follow the
// documented MATLAB behaviour (column-major double arrays, struct fields,
// mexErrMsgIdAndTxt does not return — here it throws).
#pragma once
#include <cstddef>
#include <cstdarg>
#include <string>

typedef size_t mwSize;
typedef enum { mxDOUBLE_CLASS, mxSINGLE_CLASS, mxCHAR_CLASS, mxSTRUCT_CLASS } mxClassID;
typedef enum { mxREAL, mxCOMPLEX } mxComplexity;
struct mxArray;

struct MockMexError {
    std::string id, msg;
};

bool mxIsStruct(const mxArray*);
bool mxIsDouble(const mxArray*);
bool mxIsSingle(const mxArray*);
bool mxIsComplex(const mxArray*);
bool mxIsChar(const mxArray*);
mxArray* mxGetField(const mxArray*, size_t, const char*);
double mxGetScalar(const mxArray*);
mwSize mxGetNumberOfDimensions(const mxArray*);
const mwSize* mxGetDimensions(const mxArray*);
size_t mxGetNumberOfElements(const mxArray*);
double* mxGetPr(const mxArray*);
void* mxGetData(const mxArray*);
void mxSetM(mxArray*, mwSize);
int mxGetString(const mxArray*, char*, mwSize);
mxArray* mxCreateNumericArray(mwSize, const mwSize*, mxClassID, mxComplexity);
mxArray* mxCreateDoubleMatrix(mwSize, mwSize, mxComplexity);
void mxDestroyArray(mxArray*);
void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...);
void mexWarnMsgIdAndTxt(const char* id, const char* fmt, ...);
int mexPrintf(const char* fmt, ...);
int mexAtExit(void (*fn)(void));
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]);
