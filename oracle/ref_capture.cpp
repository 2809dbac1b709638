// ref_capture.cpp -- golden-fixture capture harness around the REFERENCE code.
//
// TEST INFRASTRUCTURE ONLY (builds into oracle/_ref/, never shipped).
// It compiles the reference's own main.cpp where it lies under /root/reference
// (renaming its main) and calls the reference's KNN(), computeConfusionMatrix()
// and computeAccuracy() (main.cpp:25,87,102) on ARFF inputs parsed by the
// reference's libarff.  With a 6th argument it also records each query's top-k
// as (float bits, train index), using the reference's distance() (main.cpp:14)
// and std::stable_sort -- SURVEY.md 8c verified this equals the insertion
// queue's order (ties -> lower train index).
//
// usage: ref_capture train.arff test.arff k pred_out.txt [topk_out.bin]
//   pred_out.txt : "%d\n" per query (the sha256 contract of SURVEY.md 8c)
//   stdout       : accuracy line + confusion matrix rows
//   topk_out.bin : int32 header {nq, k}, then nq*k records {uint32 dist_bits, int32 idx}
#define main reference_main
#include REF_MAIN_CPP
#undef main

#include <algorithm>
#include <cstring>
#include <vector>

int main(int argc, char** argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s train test k pred_out [topk_out]\n", argv[0]);
        return 2;
    }
    int k = strtol(argv[3], NULL, 10);
    ArffParser parserTrain(argv[1]);
    ArffParser parserTest(argv[2]);
    ArffData* train = parserTrain.parse();
    ArffData* test = parserTest.parse();

    int* pred = KNN(train, test, k);
    FILE* f = fopen(argv[4], "w");
    for (long q = 0; q < test->num_instances(); q++) fprintf(f, "%d\n", pred[q]);
    fclose(f);

    int* cm = computeConfusionMatrix(pred, test);
    float acc = computeAccuracy(cm, test);
    long C = test->num_classes();
    printf("accuracy %.4f classes %ld\n", acc, C);
    for (long r = 0; r < C; r++) {
        for (long c = 0; c < C; c++) printf(c ? " %d" : "%d", cm[r * C + c]);
        printf("\n");
    }

    if (argc > 5 && k > 0) {
        FILE* g = fopen(argv[5], "wb");
        int32_t hdr[2] = {(int32_t)test->num_instances(), k};
        fwrite(hdr, sizeof(hdr), 1, g);
        long nt = train->num_instances();
        std::vector<std::pair<float, int32_t>> all(nt);
        for (long q = 0; q < test->num_instances(); q++) {
            for (long t = 0; t < nt; t++)
                all[t] = {distance(test->get_instance(q), train->get_instance(t)), (int32_t)t};
            std::stable_sort(all.begin(), all.end(),
                             [](const std::pair<float, int32_t>& a,
                                const std::pair<float, int32_t>& b) { return a.first < b.first; });
            for (int j = 0; j < k; j++) {
                uint32_t bits;
                std::memcpy(&bits, &all[j].first, 4);
                int32_t rec[2] = {(int32_t)bits, all[j].second};
                fwrite(rec, sizeof(rec), 1, g);
            }
        }
        fclose(g);
    }
    return 0;
}
