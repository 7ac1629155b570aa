// CLIP byte-level BPE merge loop (the per-word hot path of comfy/sd1_clip.py:360's
// transformers.CLIPTokenizer). Input words arrive already byte-encoded to printable unicode
// (Python's regex pre-tokenisation stays in Python); symbols are UTF-8 code points, the last one
// gets the "</w>" suffix, and the lowest-ranked adjacent pair is merged until none is in the merge
// table. Results are memoised per word (prompts repeat words constantly).
#include "runtime.h"

#include <climits>
#include <stdexcept>

namespace cgs {

BPE::BPE(const std::vector<std::string>& merges, const std::vector<std::string>& vocab) {
  ranks_.reserve(merges.size() * 2);
  for (size_t i = 0; i < merges.size(); ++i) ranks_.emplace(merges[i], int(i));
  encoder_.reserve(vocab.size() * 2);
  for (size_t i = 0; i < vocab.size(); ++i) encoder_.emplace(vocab[i], int(i));
}

static std::vector<std::string> split_utf8(const std::string& w) {
  std::vector<std::string> out;
  size_t i = 0;
  while (i < w.size()) {
    unsigned char c = static_cast<unsigned char>(w[i]);
    size_t n = c < 0x80 ? 1 : (c >> 5) == 0x6 ? 2 : (c >> 4) == 0xE ? 3 : 4;
    if (i + n > w.size()) n = w.size() - i;
    out.emplace_back(w.substr(i, n));
    i += n;
  }
  return out;
}

std::vector<int> BPE::bpe(const std::string& word) const {
  std::vector<std::string> sym = split_utf8(word);
  if (sym.empty()) return {};
  sym.back() += "</w>";
  std::string key;
  while (sym.size() > 1) {
    int best = INT_MAX;
    size_t bi = 0;
    for (size_t i = 0; i + 1 < sym.size(); ++i) {
      key.assign(sym[i]);
      key += ' ';
      key += sym[i + 1];
      auto it = ranks_.find(key);
      if (it != ranks_.end() && it->second < best) { best = it->second; bi = i; }
    }
    if (best == INT_MAX) break;
    // merge every occurrence of the best pair, left to right
    const std::string a = sym[bi], b = sym[bi + 1];
    std::vector<std::string> nxt;
    nxt.reserve(sym.size());
    for (size_t i = 0; i < sym.size();) {
      if (i + 1 < sym.size() && sym[i] == a && sym[i + 1] == b) {
        nxt.push_back(a + b);
        i += 2;
      } else {
        nxt.push_back(sym[i]);
        ++i;
      }
    }
    sym.swap(nxt);
  }
  std::vector<int> ids;
  ids.reserve(sym.size());
  for (auto& s : sym) {
    auto it = encoder_.find(s);
    if (it != encoder_.end()) ids.push_back(it->second);
  }
  return ids;
}

std::vector<int> BPE::encode_word(const std::string& utf8_word) {
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = cache_.find(utf8_word);
    if (it != cache_.end()) return it->second;
  }
  std::vector<int> ids = bpe(utf8_word);
  std::lock_guard<std::mutex> g(mu_);
  if (cache_.size() > 200000) cache_.clear();
  cache_.emplace(utf8_word, ids);
  return ids;
}

}  // namespace cgs
