// Diagnostic translation unit (never shipped): the product kernels with the hooks of sng_diag_hooks.h
// filled in by the -DSNG_DIAG_* flag tools/diag/Makefile passes.
#include "sng_kernels.hip"
