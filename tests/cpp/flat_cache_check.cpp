// flat_cache_check.cpp -- the C++ KNN() surface over a sequence of datasets that are parsed,
// classified and freed one after another (tests/test_gpu_host_path.py).  The device contexts
// cache the train upload (KNN_OPT_CACHE_TRAIN); a freed ArffData's pinned buffers can come
// back at the same address for the next dataset of the same shape, so the cache must be keyed
// on the flat view's unique id, not on the address.  Prints one line of predictions per pair.
//
//   flat_cache_check k train0.arff test0.arff [train1.arff test1.arff ...]
#include <cstdio>
#include <cstdlib>

#include "../../include/knn_arff.hpp"

int main(int argc, char* argv[]) {
    if (argc < 4 || (argc - 2) % 2) {
        std::fprintf(stderr, "usage: flat_cache_check k train.arff test.arff [...]\n");
        return 2;
    }
    const int k = (int)std::strtol(argv[1], nullptr, 10);
    for (int i = 2; i + 1 < argc; i += 2) {
        ArffParser* ptr = new ArffParser(argv[i]);
        ArffParser* pte = new ArffParser(argv[i + 1]);
        ArffData* train = ptr->parse();
        ArffData* test = pte->parse();
        std::fprintf(stderr, "pair %d: train feat at %p\n", i / 2, (const void*)train->flat().feat.data());
        int* pred = KNN(train, test, k);
        for (long q = 0; q < test->num_instances(); q++) std::printf(q ? " %d" : "%d", pred[q]);
        std::printf("\n");
        std::free(pred);
        delete pte;  // frees the datasets (and their pinned flat views)
        delete ptr;
    }
    return 0;
}
