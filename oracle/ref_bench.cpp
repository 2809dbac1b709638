// ref_bench.cpp -- CPU baseline: the REFERENCE pthreads KNN timed on a sample.
//
// TEST/BENCH INFRASTRUCTURE ONLY (builds into oracle/_ref/, travels to the GPU
// box as a binary; bench.py's cpu_baseline leg runs it).  It compiles the
// reference's multi-thread.cpp where it lies under /root/reference (renaming
// its main) and drives the reference's own `void* KNN(void*)` thread function
// (multi-thread.cpp:37) with the reference's partition rule
// (multi-thread.cpp:154-192: contiguous split, remainder to the last thread).
// The synthetic rows are built in memory through libarff's public API
// (ArffData::add_attr / add_instance, ArffValue(float)) instead of parsing
// ARFF text, because libarff parses at ~0.5 M values/s.
// Values come from the same counter-based generator as the GPU path
// (oracle/knn_oracle.c oracle_gen_*), so the predictions can be cross-checked.
//
// usage: ref_bench kind seed nt nq d k C threads [pred_out]
//   kind 0 = fp32 grid values, 1 = bf16-exact values, 2 / 3 = their clustered variants
// stdout: one JSON line {"ms":..,"pairs_per_s":..,"queries_per_s":..,"threads":..}
#define main reference_main
#include REF_MT_CPP
#undef main

#include <string>

extern "C" {
float oracle_gen_value_c(uint64_t seed, uint32_t stream, uint64_t row, uint32_t col, int kind, int C);
int32_t oracle_gen_label(uint64_t seed, uint32_t stream, uint64_t row, int C);
}

static ArffData* build(int kind, uint64_t seed, uint32_t stream, long n, int d, int C) {
    ArffData* data = new ArffData();
    for (int i = 0; i < d; i++) data->add_attr(new ArffAttr("A" + std::to_string(i), NUMERIC));
    data->add_attr(new ArffAttr("class", NUMERIC));
    for (long r = 0; r < n; r++) {
        ArffInstance* inst = new ArffInstance();
        for (int c = 0; c < d; c++)
            inst->add(new ArffValue(oracle_gen_value_c(seed, stream, (uint64_t)r, (uint32_t)c, kind, C)));
        inst->add(new ArffValue((float)oracle_gen_label(seed, stream, (uint64_t)r, C)));
        data->add_instance(inst);
    }
    return data;
}

int main(int argc, char** argv) {
    if (argc < 9) {
        fprintf(stderr, "usage: %s kind seed nt nq d k C threads [pred_out]\n", argv[0]);
        return 2;
    }
    int kind = atoi(argv[1]);
    uint64_t seed = strtoull(argv[2], NULL, 10);
    long nt = atol(argv[3]), nq = atol(argv[4]);
    int d = atoi(argv[5]), k = atoi(argv[6]), C = atoi(argv[7]), numThreads = atoi(argv[8]);

    ArffData* train = build(kind, seed, 0, nt, d, C);
    ArffData* test = build(kind, seed, 1, nq, d, C);
    train->num_classes();  // warm the lazy cache before fan-out (TSAN race)

    pthread_t* threads = (pthread_t*)malloc(numThreads * sizeof(pthread_t));
    int per = nq / numThreads, left = nq % numThreads;
    predictions = (int*)malloc(nq * sizeof(int));
    std::vector<arguments*> params;
    struct timespec start, end;
    clock_gettime(CLOCK_MONOTONIC_RAW, &start);
    int s = 0;
    for (int i = 0; i < numThreads; i++) {
        arguments* a = (arguments*)malloc(sizeof(arguments));
        int e = s + per + (i == numThreads - 1 ? left : 0);
        a->train = train; a->test = test; a->k = k; a->start = s; a->end = e;
        params.push_back(a);
        pthread_create(&threads[i], NULL, KNN, (void*)a);
        s = e;
    }
    for (int i = 0; i < numThreads; i++) pthread_join(threads[i], NULL);
    clock_gettime(CLOCK_MONOTONIC_RAW, &end);
    double ms = (1e9 * (end.tv_sec - start.tv_sec) + (end.tv_nsec - start.tv_nsec)) / 1e6;
    double pairs = (double)nt * (double)nq;
    printf("{\"ms\": %.3f, \"pairs_per_s\": %.6g, \"queries_per_s\": %.6g, \"threads\": %d, "
           "\"nt\": %ld, \"nq\": %ld, \"d\": %d, \"k\": %d}\n",
           ms, pairs / (ms / 1e3), nq / (ms / 1e3), numThreads, nt, nq, d, k);
    if (argc > 9) {
        FILE* f = fopen(argv[9], "w");
        for (long q = 0; q < nq; q++) fprintf(f, "%d\n", predictions[q]);
        fclose(f);
    }
    return 0;
}
