// Native host tokenizers (K18): GPT-2 byte-level BPE and BERT (uncased) WordPiece.
//
// The reference calls HF's Python GPT2Tokenizer / BertTokenizer (tutoring_server.py:11,20,30;
// lms_server.py:97-101).  These are C++ re-implementations of the same algorithms, exposed through a
// C ABI (ctypes):
//   * BPE: GPT-2's bytes->unicode table, its pre-tokenisation pattern (contractions, letter runs,
//     digit runs, punctuation runs, whitespace), rank-ordered pair merges, and byte-exact decoding.
//     Loads vocab.json + merges.txt when given; without them (no network here) it runs on a
//     synthetic vocabulary: the 256 byte tokens at GPT-2's ids 0..255, no merges, and ids >= 256
//     decoded to deterministic pseudo-words so random-init model output is still printable text.
//     Optional synthetic *word* mode (dlms_bpe_set_synthetic_words): every multi-byte pre-token
//     gets one hashed id in [256, V-1) (byte fallback on a hash collision), so prompt lengths in
//     tokens are close to real GPT-2 BPE's (~1 token per word) instead of 1 token per byte.
//   * WordPiece: BERT's basic tokenizer (lower-case, accent-strip for Latin-1, split on whitespace
//     and punctuation, CJK as single chars) + greedy longest-match-first sub-words with "##".
//     Loads vocab.txt; without it a deterministic hashed vocabulary stands in.
// Non-ASCII code points are classified as letters (no ICU on the box); exact for ASCII text.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <unordered_map>
#include <mutex>
#include <vector>

namespace {

// ------------------------------------------------------------------------------------ UTF-8
void append_utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) {
        out.push_back((char)cp);
    } else if (cp < 0x800) {
        out.push_back((char)(0xC0 | (cp >> 6)));
        out.push_back((char)(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
        out.push_back((char)(0xE0 | (cp >> 12)));
        out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
        out.push_back((char)(0x80 | (cp & 0x3F)));
    } else {
        out.push_back((char)(0xF0 | (cp >> 18)));
        out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
        out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
        out.push_back((char)(0x80 | (cp & 0x3F)));
    }
}

// decode one code point at s[i], advancing i; invalid bytes map to themselves (Latin-1)
uint32_t next_cp(const std::string& s, size_t& i) {
    unsigned char c = (unsigned char)s[i];
    int n = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
    if (n == 0 || i + n > s.size()) {
        ++i;
        return c;
    }
    uint32_t cp = n == 1 ? c : n == 2 ? (c & 0x1F) : n == 3 ? (c & 0x0F) : (c & 0x07);
    for (int k = 1; k < n; ++k) {
        unsigned char d = (unsigned char)s[i + k];
        if ((d & 0xC0) != 0x80) {
            ++i;
            return c;
        }
        cp = (cp << 6) | (d & 0x3F);
    }
    i += n;
    return cp;
}

bool is_space(uint32_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == 0x0B || c == 0x0C || c == 0xA0; }
bool is_digit(uint32_t c) { return c >= '0' && c <= '9'; }
bool is_letter(uint32_t c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c >= 0x80; }
bool is_ascii_punct(uint32_t c) {
    return (c >= 33 && c <= 47) || (c >= 58 && c <= 64) || (c >= 91 && c <= 96) || (c >= 123 && c <= 126);
}

// ------------------------------------------------------------------------------------ JSON (flat)
// Parses {"token": id, ...} -- enough for GPT-2's vocab.json.
bool parse_vocab_json(const std::string& text, std::unordered_map<std::string, int>& out) {
    size_t i = text.find('{');
    if (i == std::string::npos) return false;
    ++i;
    while (i < text.size()) {
        while (i < text.size() && (isspace((unsigned char)text[i]) || text[i] == ',')) ++i;
        if (i >= text.size() || text[i] == '}') break;
        if (text[i] != '"') return false;
        ++i;
        std::string key;
        while (i < text.size() && text[i] != '"') {
            if (text[i] == '\\' && i + 1 < text.size()) {
                char e = text[++i];
                if (e == 'u' && i + 4 < text.size()) {
                    uint32_t cp = (uint32_t)std::stoul(text.substr(i + 1, 4), nullptr, 16);
                    i += 4;
                    if (cp >= 0xD800 && cp < 0xDC00 && i + 6 < text.size() && text[i + 1] == '\\' && text[i + 2] == 'u') {
                        uint32_t lo = (uint32_t)std::stoul(text.substr(i + 3, 4), nullptr, 16);
                        cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                        i += 6;
                    }
                    append_utf8(key, cp);
                } else {
                    key.push_back(e == 'n' ? '\n' : e == 't' ? '\t' : e == 'r' ? '\r' : e == 'b' ? '\b' : e == 'f' ? '\f' : e);
                }
                ++i;
            } else {
                key.push_back(text[i++]);
            }
        }
        ++i;
        while (i < text.size() && (isspace((unsigned char)text[i]) || text[i] == ':')) ++i;
        size_t j = i;
        while (j < text.size() && (text[j] == '-' || isdigit((unsigned char)text[j]))) ++j;
        out[key] = std::stoi(text.substr(i, j - i));
        i = j;
    }
    return true;
}

std::string read_file(const char* path) {
    std::ifstream f(path, std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

// ------------------------------------------------------------------------------------ BPE
struct PairHash {
    size_t operator()(const std::pair<std::string, std::string>& p) const {
        return std::hash<std::string>()(p.first) * 1315423911u ^ std::hash<std::string>()(p.second);
    }
};

struct BPE {
    std::string byte_enc[256];                     // byte -> UTF-8 of its unicode stand-in
    std::unordered_map<uint32_t, int> byte_dec;     // stand-in code point -> byte
    std::unordered_map<std::string, int> encoder;   // token (stand-in text) -> id
    std::vector<std::string> decoder;               // id -> token
    std::unordered_map<std::pair<std::string, std::string>, int, PairHash> ranks;
    std::unordered_map<std::string, std::vector<int>> cache;
    bool synthetic = false;
    int vocab_size = 50257;
    int word_vocab = 0;                                  // synthetic word mode: model vocab size
    std::unordered_map<int, std::string> word_of;        // hashed word id -> word bytes
    std::mutex mu;                                       // ctypes drops the GIL: serialise

    BPE() {
        // GPT-2 bytes_to_unicode: printable Latin-1 bytes map to themselves, the rest to 256+n
        std::vector<int> bs;
        for (int b = '!'; b <= '~'; ++b) bs.push_back(b);
        for (int b = 0xA1; b <= 0xAC; ++b) bs.push_back(b);
        for (int b = 0xAE; b <= 0xFF; ++b) bs.push_back(b);
        std::vector<int> cs(bs);
        int n = 0;
        for (int b = 0; b < 256; ++b) {
            bool found = false;
            for (int x : bs)
                if (x == b) found = true;
            if (!found) {
                bs.push_back(b);
                cs.push_back(256 + n++);
            }
        }
        for (size_t k = 0; k < bs.size(); ++k) {
            std::string s;
            append_utf8(s, (uint32_t)cs[k]);
            byte_enc[bs[k]] = s;
            byte_dec[(uint32_t)cs[k]] = bs[k];
        }
    }

    void init_synthetic() {
        synthetic = true;
        // GPT-2's first 256 ids are the byte tokens in bytes_to_unicode order
        std::vector<int> order;
        for (int b = '!'; b <= '~'; ++b) order.push_back(b);
        for (int b = 0xA1; b <= 0xAC; ++b) order.push_back(b);
        for (int b = 0xAE; b <= 0xFF; ++b) order.push_back(b);
        for (int b = 0; b < 256; ++b) {
            bool found = false;
            for (int x : order)
                if (x == b) found = true;
            if (!found) order.push_back(b);
        }
        decoder.assign(256, "");
        for (int id = 0; id < 256; ++id) {
            decoder[id] = byte_enc[order[id]];
            encoder[decoder[id]] = id;
        }
    }

    bool load(const char* vocab_path, const char* merges_path) {
        std::string v = read_file(vocab_path);
        if (v.empty() || !parse_vocab_json(v, encoder)) return false;
        int mx = 0;
        for (auto& kv : encoder) mx = kv.second > mx ? kv.second : mx;
        decoder.assign(mx + 1, "");
        for (auto& kv : encoder) decoder[kv.second] = kv.first;
        vocab_size = mx + 1;
        std::ifstream f(merges_path);
        std::string line;
        int r = 0;
        while (std::getline(f, line)) {
            if (line.empty() || line[0] == '#') continue;
            size_t sp = line.find(' ');
            if (sp == std::string::npos) continue;
            std::string a = line.substr(0, sp), b = line.substr(sp + 1);
            while (!b.empty() && (b.back() == '\r' || b.back() == '\n')) b.pop_back();
            ranks[{a, b}] = r++;
        }
        return true;
    }

    // GPT-2 pre-tokenisation: 's|'t|'re|'ve|'m|'ll|'d| ?L+| ?N+| ?[^\sLN]+|\s+(?!\S)|\s+
    std::vector<std::string> pretokenize(const std::string& text) const {
        std::vector<uint32_t> cps;
        std::vector<size_t> offs;
        for (size_t i = 0; i < text.size();) {
            offs.push_back(i);
            cps.push_back(next_cp(text, i));
        }
        offs.push_back(text.size());
        std::vector<std::string> out;
        size_t n = cps.size(), i = 0;
        auto emit = [&](size_t a, size_t b) { out.push_back(text.substr(offs[a], offs[b] - offs[a])); };
        while (i < n) {
            uint32_t c = cps[i];
            if (c == '\'' && i + 1 < n) {
                uint32_t d = cps[i + 1] | 0x20;
                uint32_t e = i + 2 < n ? (cps[i + 2] | 0x20) : 0;
                if (cps[i + 1] == 's' || cps[i + 1] == 't' || cps[i + 1] == 'm' || cps[i + 1] == 'd') {
                    emit(i, i + 2);
                    i += 2;
                    continue;
                }
                if ((d == 'r' && e == 'e') || (d == 'v' && e == 'e') || (d == 'l' && e == 'l')) {
                    if ((cps[i + 1] == 'r' || cps[i + 1] == 'v' || cps[i + 1] == 'l')) {
                        emit(i, i + 3);
                        i += 3;
                        continue;
                    }
                }
            }
            size_t j = i;
            bool lead_space = (c == ' ' && i + 1 < n && !is_space(cps[i + 1]));
            size_t k = lead_space ? i + 1 : i;
            uint32_t h = cps[k];
            if (is_letter(h)) {
                j = k;
                while (j < n && is_letter(cps[j])) ++j;
            } else if (is_digit(h)) {
                j = k;
                while (j < n && is_digit(cps[j])) ++j;
            } else if (!is_space(h)) {
                j = k;
                while (j < n && !is_space(cps[j]) && !is_letter(cps[j]) && !is_digit(cps[j])) ++j;
            } else {
                // whitespace run: leave the last space to prefix the next word (\s+(?!\S))
                j = i;
                while (j < n && is_space(cps[j])) ++j;
                if (j < n && j - i > 1) --j;
            }
            emit(i, j);
            i = j;
        }
        return out;
    }

    std::vector<int> bpe_word(const std::string& word) {
        auto it = cache.find(word);
        if (it != cache.end()) return it->second;
        std::vector<std::string> parts;
        for (unsigned char b : word) parts.push_back(byte_enc[b]);
        if (!ranks.empty()) {
            while (parts.size() > 1) {
                int best = -1;
                size_t at = 0;
                for (size_t k = 0; k + 1 < parts.size(); ++k) {
                    auto r = ranks.find({parts[k], parts[k + 1]});
                    if (r != ranks.end() && (best < 0 || r->second < best)) {
                        best = r->second;
                        at = k;
                    }
                }
                if (best < 0) break;
                std::vector<std::string> merged;
                const std::string a = parts[at], b = parts[at + 1];
                for (size_t k = 0; k < parts.size();) {
                    if (k + 1 < parts.size() && parts[k] == a && parts[k + 1] == b) {
                        merged.push_back(a + b);
                        k += 2;
                    } else {
                        merged.push_back(parts[k++]);
                    }
                }
                parts.swap(merged);
            }
        }
        std::vector<int> ids;
        for (auto& p : parts) {
            auto e = encoder.find(p);
            if (e != encoder.end()) {
                ids.push_back(e->second);
            } else {  // unknown merged piece: fall back to its bytes
                size_t i = 0;
                while (i < p.size()) {
                    uint32_t cp = next_cp(p, i);
                    std::string s;
                    append_utf8(s, cp);
                    auto e2 = encoder.find(s);
                    if (e2 != encoder.end()) ids.push_back(e2->second);
                }
            }
        }
        if (cache.size() < 100000) cache[word] = ids;
        return ids;
    }

    int word_id(const std::string& w) {
        uint32_t h = 2166136261u;  // FNV-1a
        for (unsigned char c : w) h = (h ^ c) * 16777619u;
        const int id = 256 + (int)(h % (uint32_t)(word_vocab - 257));
        auto it = word_of.find(id);
        if (it == word_of.end()) {
            word_of.emplace(id, w);
            return id;
        }
        return it->second == w ? id : -1;
    }

    std::vector<int> encode(const std::string& text) {
        std::lock_guard<std::mutex> g(mu);
        std::vector<int> ids;
        for (auto& w : pretokenize(text)) {
            if (word_vocab > 257 && w.size() > 1) {
                const int id = word_id(w);
                if (id >= 0) {
                    ids.push_back(id);
                    continue;
                }
            }
            auto v = bpe_word(w);
            ids.insert(ids.end(), v.begin(), v.end());
        }
        return ids;
    }

    std::string synthetic_piece(int id) const {
        static const char* syl[] = {"ka", "lo", "mi", "ne", "ru", "sa", "ti", "vo", "ze", "pa", "qu", "del",
                                    "ion", "ar", "en", "or", "is", "um", "ex", "tra", "ph", "st", "ch", "ly"};
        uint32_t h = (uint32_t)id * 2654435761u;
        std::string s = " ";
        int n = 1 + (int)(h % 3);
        for (int k = 0; k < n; ++k) {
            s += syl[(h >> (5 * k + 2)) % 24];
        }
        return s;
    }

    std::string decode(const int* ids, int n) {
        std::lock_guard<std::mutex> g(mu);
        std::string bytes;
        for (int k = 0; k < n; ++k) {
            int id = ids[k];
            if (word_vocab) {
                auto w = word_of.find(id);
                if (w != word_of.end()) {
                    bytes += w->second;
                    continue;
                }
            }
            if (id >= 0 && id < (int)decoder.size() && !decoder[id].empty()) {
                const std::string& t = decoder[id];
                size_t i = 0;
                while (i < t.size()) {
                    uint32_t cp = next_cp(t, i);
                    auto d = byte_dec.find(cp);
                    if (d != byte_dec.end())
                        bytes.push_back((char)d->second);
                    else
                        append_utf8(bytes, cp);
                }
            } else if (synthetic && id >= 0 && id < vocab_size) {
                bytes += synthetic_piece(id);
            }
        }
        return bytes;
    }
};

// ------------------------------------------------------------------------------------ WordPiece
struct WordPiece {
    std::unordered_map<std::string, int> vocab;
    bool synthetic = false;
    int unk = 100, cls = 101, sep = 102, pad = 0, vocab_size = 30522;
    bool lower = true;

    bool load(const char* path) {
        std::ifstream f(path);
        if (!f) return false;
        std::string line;
        int id = 0;
        while (std::getline(f, line)) {
            while (!line.empty() && (line.back() == '\r' || line.back() == '\n')) line.pop_back();
            vocab[line] = id++;
        }
        vocab_size = id;
        auto g = [&](const char* t, int d) {
            auto it = vocab.find(t);
            return it == vocab.end() ? d : it->second;
        };
        unk = g("[UNK]", unk);
        cls = g("[CLS]", cls);
        sep = g("[SEP]", sep);
        pad = g("[PAD]", pad);
        return id > 0;
    }

    static uint32_t strip_accent(uint32_t c) {
        // Latin-1 accented letters -> base letter (NFD + drop Mn for the common block)
        static const char* map = "AAAAAAACEEEEIIIIDNOOOOOxOUUUUYPsaaaaaaaceeeeiiiidnooooo/ouuuuypy";
        if (c >= 0xC0 && c <= 0xFF) {
            char m = map[c - 0xC0];
            if (m != 'x' && m != '/' && m != 'P' && m != 'p' && m != 's' && m != 'D' && m != 'd') return (uint32_t)m;
        }
        return c;
    }

    static bool is_cjk(uint32_t c) {
        return (c >= 0x4E00 && c <= 0x9FFF) || (c >= 0x3400 && c <= 0x4DBF) || (c >= 0xF900 && c <= 0xFAFF) ||
               (c >= 0x20000 && c <= 0x2FA1F);
    }

    std::vector<std::string> basic(const std::string& text) const {
        std::vector<std::string> toks;
        std::string cur;
        auto flush = [&]() {
            if (!cur.empty()) toks.push_back(cur);
            cur.clear();
        };
        for (size_t i = 0; i < text.size();) {
            uint32_t c = next_cp(text, i);
            if (c == 0 || c == 0xFFFD || (c < 32 && !is_space(c))) continue;
            if (lower) {
                if (c >= 'A' && c <= 'Z') c += 32;
                if (c >= 0xC0 && c <= 0xDE && c != 0xD7) c += 32;
                c = strip_accent(c);
            }
            if (is_space(c)) {
                flush();
            } else if (is_ascii_punct(c) || is_cjk(c) || (c >= 0x2000 && c <= 0x206F)) {
                flush();
                std::string s;
                append_utf8(s, c);
                toks.push_back(s);
            } else {
                append_utf8(cur, c);
            }
        }
        flush();
        return toks;
    }

    int hashed_id(const std::string& piece) const {
        uint64_t h = 1469598103934665603ull;
        for (unsigned char ch : piece) h = (h ^ ch) * 1099511628211ull;
        const int base = vocab_size > 2000 ? 1000 : 110;  // above [PAD]/[UNK]/[CLS]/[SEP]/[MASK]
        return base + (int)(h % (uint64_t)(vocab_size - base));
    }

    void encode_word(const std::string& w, std::vector<int>& out) const {
        if (synthetic) {
            // hashed "sub-words" of up to 4 characters keep sequence lengths WordPiece-like
            size_t i = 0;
            bool first = true;
            while (i < w.size()) {
                size_t j = i;
                int cnt = 0;
                while (j < w.size() && cnt < 4) {
                    next_cp(w, j);
                    ++cnt;
                }
                out.push_back(hashed_id((first ? "" : "##") + w.substr(i, j - i)));
                first = false;
                i = j;
            }
            return;
        }
        if (w.size() > 200) {
            out.push_back(unk);
            return;
        }
        std::vector<int> sub;
        size_t start = 0;
        while (start < w.size()) {
            size_t end = w.size();
            int found = -1;
            while (start < end) {
                std::string piece = (start > 0 ? "##" : "") + w.substr(start, end - start);
                auto it = vocab.find(piece);
                if (it != vocab.end()) {
                    found = it->second;
                    break;
                }
                // step back one UTF-8 code point
                do {
                    --end;
                } while (end > start && ((unsigned char)w[end] & 0xC0) == 0x80);
            }
            if (found < 0) {
                out.push_back(unk);
                return;
            }
            sub.push_back(found);
            start = end;
        }
        out.insert(out.end(), sub.begin(), sub.end());
    }

    std::vector<int> encode(const std::string& text, int max_len, bool special) const {
        std::vector<int> ids;
        if (special) ids.push_back(cls);
        for (auto& w : basic(text)) encode_word(w, ids);
        if (special) {
            if (max_len > 1 && (int)ids.size() > max_len - 1) ids.resize(max_len - 1);
            ids.push_back(sep);
        } else if (max_len > 0 && (int)ids.size() > max_len) {
            ids.resize(max_len);
        }
        return ids;
    }
};

int copy_out(const std::vector<int>& v, int* out, int cap) {
    int n = (int)v.size();
    if (out != nullptr) std::memcpy(out, v.data(), sizeof(int) * (size_t)(n < cap ? n : cap));
    return n;
}

}  // namespace

extern "C" {

void* dlms_bpe_create(const char* vocab_json, const char* merges_txt) {
    BPE* b = new BPE();
    if (vocab_json && merges_txt && vocab_json[0] && merges_txt[0]) {
        if (!b->load(vocab_json, merges_txt)) {
            delete b;
            return nullptr;
        }
    } else {
        b->init_synthetic();
    }
    return b;
}

int dlms_bpe_is_synthetic(void* h) { return static_cast<BPE*>(h)->synthetic ? 1 : 0; }

int dlms_bpe_vocab_size(void* h) { return static_cast<BPE*>(h)->vocab_size; }

// synthetic vocabularies only: one hashed id per word, ids < vocab (the model's vocabulary;
// id vocab-1 is left to <|endoftext|>).  Returns 0 on success.
int dlms_bpe_set_synthetic_words(void* h, int vocab) {
    BPE* b = static_cast<BPE*>(h);
    if (!b->synthetic || vocab <= 512) return -1;
    std::lock_guard<std::mutex> g(b->mu);
    b->word_vocab = vocab;
    b->vocab_size = vocab;
    b->word_of.clear();
    return 0;
}

// returns the number of ids (may exceed cap: call again with a larger buffer)
int dlms_bpe_encode(void* h, const char* text, int len, int* out, int cap) {
    return copy_out(static_cast<BPE*>(h)->encode(std::string(text, (size_t)len)), out, cap);
}

int dlms_bpe_decode(void* h, const int* ids, int n, char* out, int cap) {
    std::string s = static_cast<BPE*>(h)->decode(ids, n);
    if (out != nullptr) std::memcpy(out, s.data(), (size_t)((int)s.size() < cap ? (int)s.size() : cap));
    return (int)s.size();
}

void dlms_bpe_destroy(void* h) { delete static_cast<BPE*>(h); }

void* dlms_wp_create(const char* vocab_txt, int vocab_size) {
    WordPiece* w = new WordPiece();
    if (vocab_txt && vocab_txt[0]) {
        if (!w->load(vocab_txt)) {
            delete w;
            return nullptr;
        }
    } else {
        w->synthetic = true;
        if (vocab_size > 200) w->vocab_size = vocab_size;
    }
    return w;
}

int dlms_wp_encode(void* h, const char* text, int len, int max_len, int special, int* out, int cap) {
    return copy_out(static_cast<WordPiece*>(h)->encode(std::string(text, (size_t)len), max_len, special != 0), out,
                    cap);
}

int dlms_wp_special(void* h, int which) {
    WordPiece* w = static_cast<WordPiece*>(h);
    return which == 0 ? w->pad : which == 1 ? w->cls : which == 2 ? w->sep : w->unk;
}

void dlms_wp_destroy(void* h) { delete static_cast<WordPiece*>(h); }

}  // extern "C"
