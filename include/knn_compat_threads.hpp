// knn_compat_threads.hpp -- drop-in for the pthreads driver's KNN thread body.
//
// multi-thread.cpp:15-24,37 declares a global `int* predictions`, a
// `struct arguments {train, test, k, start, end}` and `void* KNN(void*)` that writes
// predictions[start..end).  A caller that keeps that driver includes this header
// instead of defining KNN itself; each thread's slice then runs on the GPU.
// (libknn_amd defines `predictions` weakly, so the driver's own definition wins.)
#ifndef KNN_COMPAT_THREADS_HPP
#define KNN_COMPAT_THREADS_HPP

#include "knn_arff.hpp"

extern int* predictions;  // multi-thread.cpp:15

struct arguments {        // multi-thread.cpp:18-24
    ArffData* train;
    ArffData* test;
    int k;
    int start;
    int end;
};

void* KNN(void* params);  // multi-thread.cpp:37

#endif  // KNN_COMPAT_THREADS_HPP
