// Host-side sanitizer harness for the native tokenizers (sanitizers run on host
// code only -- no GPU ASan on this pool).  Built twice by tests/test_native_sanitizers.py:
//   -fsanitize=address,undefined  round trips over random byte strings (UTF-8 and not), long
//                                 inputs, buffer-size renegotiation of the C ABI
//   -fsanitize=thread             8 threads encoding/decoding through ONE shared handle, the way
//                                 gRPC worker threads share the tutoring server's tokenizer
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

extern "C" {
void* dlms_bpe_create(const char*, const char*);
int dlms_bpe_set_synthetic_words(void*, int);
int dlms_bpe_encode(void*, const char*, int, int*, int);
int dlms_bpe_decode(void*, const int*, int, char*, int);
void dlms_bpe_destroy(void*);
void* dlms_wp_create(const char*, int);
int dlms_wp_encode(void*, const char*, int, int, int, int*, int);
void dlms_wp_destroy(void*);
}

static std::string random_text(std::mt19937& rng, int n, bool ascii) {
    static const char* words[] = {"raft", " consensus", " leader", " term", "'s", " 123", "  ", "\n", "!?", " Ünï",
                                  " 日本", "tab\t", " x"};
    std::string s;
    while ((int)s.size() < n) {
        if (ascii || rng() % 4) {
            s += words[rng() % (ascii ? 7 : 13)];
        } else {
            s.push_back((char)(rng() % 256));  // arbitrary bytes, incl. invalid UTF-8
        }
    }
    return s;
}

static int roundtrip(void* bpe, const std::string& s) {
    std::vector<int> ids(4);  // deliberately small: exercise the "call again with a bigger buffer" path
    int n = dlms_bpe_encode(bpe, s.data(), (int)s.size(), ids.data(), (int)ids.size());
    if (n > (int)ids.size()) {
        ids.resize(n);
        n = dlms_bpe_encode(bpe, s.data(), (int)s.size(), ids.data(), n);
    }
    std::vector<char> out(8);
    int m = dlms_bpe_decode(bpe, ids.data(), n, out.data(), (int)out.size());
    if (m > (int)out.size()) {
        out.resize(m);
        m = dlms_bpe_decode(bpe, ids.data(), n, out.data(), m);
    }
    return std::string(out.data(), m) == s ? 0 : 1;
}

int main(int argc, char** argv) {
    const bool threads = argc > 1 && std::strcmp(argv[1], "threads") == 0;
    void* bpe = dlms_bpe_create(nullptr, nullptr);
    void* words = dlms_bpe_create(nullptr, nullptr);
    dlms_bpe_set_synthetic_words(words, 50257);
    void* wp = dlms_wp_create(nullptr, 30522);
    int bad = 0;
    if (!threads) {
        std::mt19937 rng(7);
        for (int i = 0; i < 300; ++i) {
            const std::string s = random_text(rng, 1 + (int)(rng() % 600), false);
            bad += roundtrip(bpe, s);
            std::vector<int> ids(600);
            dlms_wp_encode(wp, s.data(), (int)s.size(), 512, 1, ids.data(), (int)ids.size());
        }
        for (int i = 0; i < 100; ++i) bad += roundtrip(words, random_text(rng, 1 + (int)(rng() % 400), true));
        const std::string big = random_text(rng, 200000, false);
        bad += roundtrip(bpe, big);
    } else {
        std::vector<std::thread> ts;
        std::vector<int> errs(8, 0);
        for (int t = 0; t < 8; ++t) {
            ts.emplace_back([&, t] {
                std::mt19937 rng(100 + t);
                for (int i = 0; i < 200; ++i) {
                    errs[t] += roundtrip(words, random_text(rng, 1 + (int)(rng() % 200), true));
                    errs[t] += roundtrip(bpe, random_text(rng, 1 + (int)(rng() % 200), false));
                    std::vector<int> ids(300);
                    const std::string s = random_text(rng, 100, true);
                    dlms_wp_encode(wp, s.data(), (int)s.size(), 256, 1, ids.data(), (int)ids.size());
                }
            });
        }
        for (auto& th : ts) th.join();
        for (int e : errs) bad += e;
    }
    dlms_bpe_destroy(bpe);
    dlms_bpe_destroy(words);
    dlms_wp_destroy(wp);
    std::printf("%s roundtrip failures: %d\n", threads ? "threads" : "single", bad);
    return bad ? 1 : 0;
}
