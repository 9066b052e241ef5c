// Native text pre-processing pipeline (host C++, OpenMP) for the IMDB classifier path.
//
// Replaces, in one multithreaded pass over all reviews, the reference's Python-loop pipeline
// (pytorch_on_language_distr.py:34-103):
//   rm_tags (regex '<[^>]+>' -> ' ')  ->  BertTokenizer(do_lower_case=True).encode(
//   add_special_tokens=True, max_length=128) (BasicTokenizer: lower-case, whitespace +
//   punctuation split; WordPiece greedy longest-match-first with '##' continuations,
//   100-char word limit -> [UNK]) -> pad_sequences(maxlen=128, padding='post',
//   truncating='post', value=0) -> attention_mask = int(token_id > 0).
// The reference tokenises every review in a single-threaded Python loop on every rank; here each
// rank runs it once at native speed across all cores.
//
// Exposed as torch.ops.pcmp.text_encode(str[] texts, str[] vocab, int max_len, bool lower,
// bool strip_tags) -> [ids int64 [N,max_len], mask int64 [N,max_len]] and
// torch.ops.pcmp.text_basic_tokenize(str[] texts, bool lower, bool strip_tags) -> str[] (space-
// joined basic tokens, used to build a vocabulary when no vocab file is available offline).
#include <torch/extension.h>

#include <string>
#include <vector>

#include "runtime/text_core.h"

namespace pcmp_rt {

std::vector<at::Tensor> text_encode(const std::vector<std::string>& texts, const std::vector<std::string>& vocab,
                                    int64_t max_len, bool lower, bool strip) {
  TORCH_CHECK(max_len >= 2, "text_encode: max_len >= 2");
  Vocab v;
  v.map.reserve(vocab.size() * 2);
  for (size_t i = 0; i < vocab.size(); ++i) v.map.emplace(vocab[i], (int64_t)i);
  auto get = [&](const char* t, int64_t d) { auto it = v.map.find(t); return it == v.map.end() ? d : it->second; };
  v.unk = get("[UNK]", 100);
  v.cls = get("[CLS]", 101);
  v.sep = get("[SEP]", 102);
  const int64_t N = (int64_t)texts.size();
  auto ids = at::zeros({N, max_len}, at::kLong);
  auto mask = at::zeros({N, max_len}, at::kLong);
  int64_t* ip = ids.data_ptr<int64_t>();
  int64_t* mp = mask.data_ptr<int64_t>();
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t n = 0; n < N; ++n) encode_row(texts[n], v, max_len, lower, strip, ip + n * max_len, mp + n * max_len);
  return {ids, mask};
}

std::vector<std::string> text_basic_tokenize(const std::vector<std::string>& texts, bool lower, bool strip) {
  std::vector<std::string> out(texts.size());
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t n = 0; n < (int64_t)texts.size(); ++n) {
    std::vector<std::string> toks;
    basic_tokenize(strip ? strip_tags(texts[n]) : texts[n], lower, toks);
    std::string s;
    for (size_t i = 0; i < toks.size(); ++i) {
      if (i) s.push_back(' ');
      s += toks[i];
    }
    out[n] = std::move(s);
  }
  return out;
}

}  // namespace pcmp_rt

TORCH_LIBRARY_FRAGMENT(pcmp, m) {
  m.def("text_encode(str[] texts, str[] vocab, int max_len, bool lower, bool strip_tags) -> Tensor[]",
        &pcmp_rt::text_encode);
  m.def("text_basic_tokenize(str[] texts, bool lower, bool strip_tags) -> str[]", &pcmp_rt::text_basic_tokenize);
}
