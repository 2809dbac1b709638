// ref_bench_mpi.cpp -- CPU baseline: the REFERENCE MPI KNN timed on a sample.
//
// TEST/BENCH INFRASTRUCTURE ONLY (builds into oracle/_ref/ against the image's MPICH,
// bench.py's cpu_baseline "mpi" leg runs it under mpiexec).  It compiles the reference's
// mpi.cpp where it lies under /root/reference (renaming its main) and drives the
// reference's own `int* KNN(ArffData*, ArffData*, int k, int start, int end)`
// (mpi.cpp:26) with the reference's scatter / gather pattern (mpi.cpp:141-186: rank 0
// computes [start, end) pairs, MPI_Scatter, per-rank KNN, MPI_Gatherv at displacement
// rank * dataPerProcess), timed from before the scatter to after the gather as
// mpi.cpp:157/189 do.  Rows come from the same generator as ref_bench.cpp (built in
// memory through libarff's API: libarff's parser is too slow for 1e5-row samples).
//
// usage: mpiexec -n N ref_bench_mpi kind seed nt nq d k C [pred_out]
// stdout (rank 0): one JSON line {"ms":..,"pairs_per_s":..,"queries_per_s":..,"ranks":..}
#define main reference_main
#include REF_MPI_CPP
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
    MPI_Init(&argc, &argv);
    int rank, world;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &world);
    if (argc < 8) {
        if (rank == 0) fprintf(stderr, "usage: %s kind seed nt nq d k C [pred_out]\n", argv[0]);
        MPI_Finalize();
        return 2;
    }
    int kind = atoi(argv[1]);
    uint64_t seed = strtoull(argv[2], NULL, 10);
    long nt = atol(argv[3]), nq = atol(argv[4]);
    int d = atoi(argv[5]), k = atoi(argv[6]), C = atoi(argv[7]);
    ArffData* train = build(kind, seed, 0, nt, d, C);
    ArffData* test = build(kind, seed, 1, nq, d, C);
    train->num_classes();
    MPI_Barrier(MPI_COMM_WORLD);  // every rank has its copy (mpi.cpp parses before t0 too)

    int per = (int)nq / world, last = per + (int)nq % world;
    std::vector<int> spans(2 * world), counts(world), displs(world);
    int mine[2];
    struct timespec t0, t1;
    if (rank == 0) {
        clock_gettime(CLOCK_MONOTONIC_RAW, &t0);
        int s = 0;
        for (int i = 0; i < world; i++) {
            int e = s + (i < world - 1 ? per : last);
            spans[2 * i] = s;
            spans[2 * i + 1] = e;
            s = e;
        }
    }
    MPI_Scatter(spans.data(), 2, MPI_INT, mine, 2, MPI_INT, 0, MPI_COMM_WORLD);
    int* sub = KNN(train, test, k, mine[0], mine[1]);
    for (int i = 0; i < world; i++) {
        counts[i] = i < world - 1 ? per : last;
        displs[i] = i * per;
    }
    std::vector<int> pred(rank == 0 ? nq : 1);
    MPI_Gatherv(sub, rank < world - 1 ? per : last, MPI_INT, pred.data(), counts.data(), displs.data(), MPI_INT, 0,
                MPI_COMM_WORLD);
    if (rank == 0) {
        clock_gettime(CLOCK_MONOTONIC_RAW, &t1);
        double ms = (1e9 * (t1.tv_sec - t0.tv_sec) + (t1.tv_nsec - t0.tv_nsec)) / 1e6;
        double pairs = (double)nt * (double)nq;
        printf("{\"ms\": %.3f, \"pairs_per_s\": %.6g, \"queries_per_s\": %.6g, \"ranks\": %d, "
               "\"nt\": %ld, \"nq\": %ld, \"d\": %d, \"k\": %d}\n",
               ms, pairs / (ms / 1e3), nq / (ms / 1e3), world, nt, nq, d, k);
        if (argc > 8) {
            FILE* f = fopen(argv[8], "w");
            for (long q = 0; q < nq; q++) fprintf(f, "%d\n", pred[q]);
            fclose(f);
        }
    }
    MPI_Finalize();
    return 0;
}
