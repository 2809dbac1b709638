// knn_arff.hpp -- the reference's C++ API surface, re-implemented on the MI355X path.
//
// A caller of srna99/KNN-using-p_threads-and-MPI keeps its code: the libarff read API
// (ArffParser / ArffData / ArffInstance / ArffValue / ArffAttr, libarff/*.h), the
// entry point `int* KNN(ArffData*, ArffData*, int)` (main.cpp:25) and the evaluation
// functions computeConfusionMatrix / computeAccuracy (main.cpp:87,102) have the same
// names, argument meaning, ownership (malloc'd results, caller frees) and error
// behaviour (std::runtime_error where libarff throws).  Behind them the dataset is
// held flat (row-major float) and KNN() runs on gfx950 through the C ABI knn_amd.h.
//
// Differences, all documented in INTEGRATION.md:
//  * KNN() throws std::runtime_error for k > n_train (the reference segfaults) and for
//    labels outside [0, num_classes); k <= 0 still yields all-zero predictions.
//  * num_classes() is computed once at parse time (no lazy-cache data race).
//  * Test queries are sharded over the visible GPUs with the reference's rule
//    (contiguous, remainder to the last worker; multi-thread.cpp:154-158).
#ifndef KNN_ARFF_HPP
#define KNN_ARFF_HPP

#include <cstddef>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "knn_amd.h"

typedef long int int32;   // libarff/arff_utils.h:16 (8 bytes on LP64, as in the reference)
typedef long long int64;  // libarff/arff_utils.h:18

enum ArffValueEnum { INTEGER = 0, FLOAT, DATE, STRING, NUMERIC, NOMINAL, UNKNOWN_VAL };
std::string arff_value2str(ArffValueEnum e);

// libarff/arff_value.h:45
class ArffValue {
public:
    ArffValue(int32 i = 0);
    ArffValue(float f);
    ArffValue(const std::string& str);  // numeric parse like libarff (FLOAT, else STRING)
    ArffValue(const std::string& str, ArffValueEnum type);
    ArffValue(ArffValueEnum type);      // a missing value of `type`
    void set(int32 i);
    void set(float f);
    void set(const std::string& str, ArffValueEnum e = STRING);
    bool missing() const;
    ArffValueEnum type() const;
    operator int32() const;        // libarff/arff_value.cpp:101
    operator float() const;        // libarff/arff_value.cpp:114
    operator std::string() const;
private:
    float m_float;
    int32 m_int;
    ArffValueEnum m_type;
    bool m_missing;
    std::string m_str;
};

// libarff/arff_attr.h:17
class ArffAttr {
public:
    ArffAttr(const std::string& name, ArffValueEnum type);
    std::string name() const;
    ArffValueEnum type() const;
private:
    std::string m_name;
    ArffValueEnum m_enum;
};

// libarff/arff_instance.h:18
class ArffInstance {
public:
    ArffInstance();
    ~ArffInstance();
    int32 size() const;
    void add(ArffValue* val);           // takes ownership
    ArffValue* get(int idx) const;      // throws on out-of-range (libarff/arff_instance.cpp:24)
private:
    std::vector<ArffValue*> m_data;
};

// Page-locked host storage for the flat view (knn_alloc_pinned), so KNN()'s uploads run as
// asynchronous DMA; plain heap memory when no device can pin it.  A 16-byte header records
// which allocator owns the block.
template <typename T>
struct KnnPinnedAllocator {
    typedef T value_type;
    KnnPinnedAllocator() = default;
    template <typename U>
    KnnPinnedAllocator(const KnnPinnedAllocator<U>&) {}
    T* allocate(size_t n) {
        void* p = nullptr;
        const size_t bytes = n * sizeof(T) + 16;
        bool pinned = knn_alloc_pinned(bytes, &p) == KNN_OK && p;
        if (!pinned) p = ::operator new(bytes);
        *static_cast<int*>(p) = pinned ? 1 : 0;
        return reinterpret_cast<T*>(static_cast<char*>(p) + 16);
    }
    void deallocate(T* t, size_t) {
        char* p = reinterpret_cast<char*>(t) - 16;
        if (*reinterpret_cast<int*>(p)) knn_free_pinned(p);
        else ::operator delete(p);
    }
    template <typename U>
    bool operator==(const KnnPinnedAllocator<U>&) const { return true; }
    template <typename U>
    bool operator!=(const KnnPinnedAllocator<U>&) const { return false; }
};

// a process-unique id per flat view (knn_arff.cpp): the device contexts key their train
// cache on it, never on an address the allocator can hand out again
uint64_t knn_flat_view_uid();

// Flat, KNN-ready view of a dataset (features [n][ld] row-major, ld = d rounded up to 4).
struct KnnFlatView {
    uint64_t uid = knn_flat_view_uid();
    std::vector<float, KnnPinnedAllocator<float>> feat;
    std::vector<int32_t, KnnPinnedAllocator<int32_t>> labels;   // (int)(float) of the class attribute (main.cpp:66)
    int64_t n = 0;
    int d = 0;
    int ld = 0;
};

// libarff/arff_data.h:27
class ArffData {
public:
    ArffData();
    ~ArffData();
    void set_relation_name(const std::string& name);
    std::string get_relation_name() const;
    int32 num_attributes() const;
    int32 num_classes();                // max class label + 1 (libarff/arff_data.cpp:41)
    void add_attr(ArffAttr* attr);      // takes ownership
    ArffAttr* get_attr(int32 idx) const;
    int32 num_instances() const;
    void add_instance(ArffInstance* inst);  // takes ownership; cross-checked like libarff
    ArffInstance* get_instance(int32 idx) const;
    void add_nominal_val(const std::string& name, const std::string& val);
    std::vector<std::string> get_nominal(const std::string& name);

    // New: the flat view KNN() hands to the device (built once, thread-safe).
    const KnnFlatView& flat() const;

private:
    friend class ArffParser;
    void cross_check(const ArffInstance* inst);
    std::string m_rel;
    std::vector<ArffAttr*> m_attrs;
    std::vector<ArffInstance*> m_instances;
    std::map<std::string, std::vector<std::string>> m_nominals;
    int32 m_num_classes = -1;
    mutable std::once_flag m_flat_once;
    mutable std::unique_ptr<KnnFlatView> m_flat;
};

// libarff/arff_parser.h -- parse() returns a dataset owned by the parser.
class ArffParser {
public:
    ArffParser(const std::string& file);
    ~ArffParser();
    ArffData* parse();
private:
    std::string m_file;
    ArffData* m_data;
};

// main.cpp:25 -- malloc'd int[test->num_instances()], caller frees.
int* KNN(ArffData* train, ArffData* test, int k);
// mpi.cpp:26 -- predictions for test rows [start, end), malloc'd int[end-start].
int* KNN(ArffData* train, ArffData* test, int k, int start, int end);
// main.cpp:87 -- calloc'd int[C*C], C = dataset->num_classes(), row = true class.
int* computeConfusionMatrix(int* predictions, ArffData* dataset);
// main.cpp:102
float computeAccuracy(int* confusionMatrix, ArffData* dataset);

// Number of GPUs KNN() shards over (env KNN_AMD_DEVICES, default: all visible).  The
// partition over them: env KNN_AMD_SHARD = test (default, the reference's split of the test
// set, train replicated), train (train rows split by the same rule, per-shard exact top-k
// merged on device 0 by (distance, global index)) or auto (knn_shard_policy).
int knn_amd_num_devices();
// Create the device contexts up front (the CLI does this before its timed region,
// as the reference parses and MPI_Init()s before starting its clock).
void knn_amd_init();

#endif  // KNN_ARFF_HPP
