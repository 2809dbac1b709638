// dropin_tap.cpp -- TEST INFRASTRUCTURE ONLY: a link-time tap for the drop-in drivers.
//
// The patched reference drivers (oracle/dropin.py) print only their accuracy line.  They
// are linked with -Wl,--wrap=<computeConfusionMatrix(int*, ArffData*)>, so their call
// main.cpp:133 / multi-thread.cpp:196 / mpi.cpp:192 lands here first: when
// KNN_DROPIN_PRED_OUT names a file, the predictions the driver got from libknn_amd's KNN
// are written to it ("%d\n" per row, the golden files' format), then the library's
// computeConfusionMatrix runs as usual.  The library itself carries no such hook.
#include <cstdio>
#include <cstdlib>

#include "knn_arff.hpp"

extern "C" int* __real__Z22computeConfusionMatrixPiP8ArffData(int* pred, ArffData* data);

extern "C" int* __wrap__Z22computeConfusionMatrixPiP8ArffData(int* pred, ArffData* data) {
    if (const char* path = std::getenv("KNN_DROPIN_PRED_OUT")) {
        if (FILE* f = std::fopen(path, "w")) {
            for (int32 i = 0; i < data->num_instances(); i++) std::fprintf(f, "%d\n", pred[i]);
            std::fclose(f);
        }
    }
    return __real__Z22computeConfusionMatrixPiP8ArffData(pred, data);
}
