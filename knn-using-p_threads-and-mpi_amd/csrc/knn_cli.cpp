// knn_cli.cpp -- command-line driver with the reference's contract.
//
//   knn_cli train.arff test.arff k [numDevices] [--shard=test|train|auto]
//
// Same positional arguments as ./main (main.cpp:114-122; k parsed with strtol) plus the
// optional worker count of ./multi-thread (multi-thread.cpp:135-143), here the number of
// GPUs the work is split over: the test set by the reference's rule (default), or
// --shard=train the train set (per-shard top-k merged), --shard=auto knn_shard_policy.  The timed region is the reference's: the KNN()
// call only (main.cpp:133-137), after parsing and device initialisation.  The report
// line is printed verbatim (main.cpp:146), "CPU time" wording included.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <iostream>
#include <string>

#include "../../include/knn_arff.hpp"

int main(int argc, char* argv[]) {
    // --shard=... may sit anywhere; the rest are the reference's positional arguments
    int n = 0;
    for (int i = 0; i < argc; i++) {
        if (!std::strncmp(argv[i], "--shard=", 8)) setenv("KNN_AMD_SHARD", argv[i] + 8, 1);
        else argv[n++] = argv[i];
    }
    argc = n;
    if (argc != 4 && argc != 5) {
        std::cout << "Usage: ./knn_cli datasets/train.arff datasets/test.arff k [numDevices] [--shard=test|train|auto]"
                  << std::endl;
        std::exit(0);
    }
    int k = (int)std::strtol(argv[3], NULL, 10);
    if (argc == 5) setenv("KNN_AMD_DEVICES", argv[4], 1);

    ArffParser parserTrain(argv[1]);
    ArffParser parserTest(argv[2]);
    ArffData* train = parserTrain.parse();
    ArffData* test = parserTest.parse();
    knn_amd_init();

    struct timespec start, end;
    clock_gettime(CLOCK_MONOTONIC_RAW, &start);
    int* predictions = KNN(train, test, k);
    clock_gettime(CLOCK_MONOTONIC_RAW, &end);

    int* confusionMatrix = computeConfusionMatrix(predictions, test);
    float accuracy = computeAccuracy(confusionMatrix, test);
    uint64_t diff = (1000000000L * (end.tv_sec - start.tv_sec) + end.tv_nsec - start.tv_nsec) / 1e6;
    printf("The %i-NN classifier for %lu test instances on %lu train instances required %llu ms CPU time. Accuracy was %.4f\n",
           k, (unsigned long)test->num_instances(), (unsigned long)train->num_instances(),
           (long long unsigned int)diff, accuracy);
    if (const char* p = std::getenv("KNN_CLI_PRED_OUT")) {  // test hook: dump predictions
        FILE* f = std::fopen(p, "w");
        for (long q = 0; q < test->num_instances(); q++) std::fprintf(f, "%d\n", predictions[q]);
        std::fclose(f);
    }
    std::free(predictions);
    std::free(confusionMatrix);
    return 0;
}
