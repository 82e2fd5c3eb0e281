// Splitter registry — repo/splitter/splitter.go:8-89.
//
// The reference keeps an unexported name -> Factory map (`splitterFactories`,
// :50-81) and exposes SupportedAlgorithms (:32-42, sorted), GetFactory (:84-86)
// and DefaultAlgorithm (:89).  Names are persisted in repository configs and
// policies, so this table must list exactly the reference's 23 names with the
// same parameters; new names must never be introduced.
#include <cstring>
#include <deque>
#include <mutex>
#include <string>

#include "kcdc_internal.h"

namespace kcdc {
namespace {

constexpr uint64_t KiB = 1024, MiB = 1024 * 1024;

// Sorted by std::strcmp order == Go sort.Strings order (byte-wise).
const Algo kAlgos[] = {
    {"DYNAMIC", kBuzhash, false, 4 * MiB},  // splitter.go:80 (legacy name, not pooled)
    {"DYNAMIC-128K-BUZHASH", kBuzhash, true, 128 * KiB},
    {"DYNAMIC-128K-RABINKARP", kRabinKarp, true, 128 * KiB},
    {"DYNAMIC-1M-BUZHASH", kBuzhash, true, 1 * MiB},
    {"DYNAMIC-1M-RABINKARP", kRabinKarp, true, 1 * MiB},
    {"DYNAMIC-256K-BUZHASH", kBuzhash, true, 256 * KiB},
    {"DYNAMIC-256K-RABINKARP", kRabinKarp, true, 256 * KiB},
    {"DYNAMIC-2M-BUZHASH", kBuzhash, true, 2 * MiB},
    {"DYNAMIC-2M-RABINKARP", kRabinKarp, true, 2 * MiB},
    {"DYNAMIC-4M-BUZHASH", kBuzhash, true, 4 * MiB},
    {"DYNAMIC-4M-RABINKARP", kRabinKarp, true, 4 * MiB},
    {"DYNAMIC-512K-BUZHASH", kBuzhash, true, 512 * KiB},
    {"DYNAMIC-512K-RABINKARP", kRabinKarp, true, 512 * KiB},
    {"DYNAMIC-8M-BUZHASH", kBuzhash, true, 8 * MiB},
    {"DYNAMIC-8M-RABINKARP", kRabinKarp, true, 8 * MiB},
    {"FIXED", kFixed, false, 4 * MiB},  // splitter.go:76 (legacy name, not pooled)
    {"FIXED-128K", kFixed, true, 128 * KiB},
    {"FIXED-1M", kFixed, true, 1 * MiB},
    {"FIXED-256K", kFixed, true, 256 * KiB},
    {"FIXED-2M", kFixed, true, 2 * MiB},
    {"FIXED-4M", kFixed, true, 4 * MiB},
    {"FIXED-512K", kFixed, true, 512 * KiB},
    {"FIXED-8M", kFixed, true, 8 * MiB},
};
constexpr int kNumAlgos = sizeof(kAlgos) / sizeof(kAlgos[0]);

thread_local std::string t_error;

// Interned custom parameterisations (kcdc_custom_algorithm); never freed so the
// returned names and Algo pointers stay valid for the life of the process.
std::mutex g_custom_mu;
std::deque<std::string> g_custom_names;
std::deque<Algo> g_custom;

}  // namespace

const Algo* find_algo(const char* name) {
    if (!name) return nullptr;
    for (const Algo& a : kAlgos)
        if (std::strcmp(a.name, name) == 0) return &a;
    std::lock_guard<std::mutex> lk(g_custom_mu);
    for (const Algo& a : g_custom)
        if (std::strcmp(a.name, name) == 0) return &a;
    return nullptr;
}

const Algo* custom_algo(int32_t kind, uint64_t avg) {
    if (kind != kFixed && kind != kBuzhash && kind != kRabinKarp) return nullptr;
    if (kind == kFixed ? avg < 1 : (avg < 2 || (avg & (avg - 1)) != 0 || avg > (uint64_t(1) << 31))) return nullptr;
    static const char* kKindName[] = {"fixed", "buzhash", "rabinkarp"};
    const std::string nm = std::string("kcdc:") + kKindName[kind] + ":" + std::to_string(avg);
    std::lock_guard<std::mutex> lk(g_custom_mu);
    for (const Algo& a : g_custom)
        if (nm == a.name) return &a;
    g_custom_names.push_back(nm);
    g_custom.push_back(Algo{g_custom_names.back().c_str(), static_cast<Kind>(kind), false, avg});
    return &g_custom.back();
}

int algo_index(const Algo* a) {
    const ptrdiff_t i = a - kAlgos;
    return (i >= 0 && i < kNumAlgos) ? static_cast<int>(i) : -1;
}
int algo_count() { return kNumAlgos; }
const Algo& algo_at(int i) { return kAlgos[i]; }

int set_error(int code, const std::string& msg) {
    t_error = msg;
    return code;
}
const char* last_error_cstr() { return t_error.c_str(); }

}  // namespace kcdc
