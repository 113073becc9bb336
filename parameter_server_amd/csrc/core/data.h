// Data ingestion: text example parsers, files (plain / gzip / HDFS), RecordIO.
//
// Reference: ExampleParser (src/data/text_parser.cc:14-250) parses one line into
// an Example{Slot{id, key[], val[]}} with slot 0 holding the label; formats
// LIBSVM, ADFEA, TERAFEA and the PS DENSE/SPARSE/SPARSE_BINARY format.
// InfoParser (src/data/info_parser.cc) accumulates per-slot statistics.
// Here a whole buffer is parsed (multi-threaded over line-aligned chunks)
// straight into a CSR minibatch (labels, row_ptr, keys, vals, slot ids), which is
// the layout the GPU localisation kernels consume. CRITEO (Criteo TSV) is added.
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace pscore {

enum class TextFormat : int {
  DENSE = 1, SPARSE = 2, SPARSE_BINARY = 3, ADFEA = 4, LIBSVM = 5, TERAFEA = 6, VW = 7,
  CRITEO = 8
};

struct SlotStat {
  uint64_t min_key = ~0ull, max_key = 0, nnz_ele = 0, nnz_ex = 0;
  int format = 0;  // SlotInfo::Format 1 DENSE 2 SPARSE 3 SPARSE_BINARY
};

struct ParseOptions {
  TextFormat format = TextFormat::LIBSVM;
  bool ignore_fea_slot = false;
  bool shuffle_fea_id = false;  // TERAFEA: murmur3 shuffle (reference --shuffle_fea_id)
  uint64_t hash_mod = 0;        // every key mod this (the hashing trick; 0 = none)
  int nthreads = 1;
  int64_t max_lines = -1;
};

struct ParsedBatch {
  std::vector<float> labels;
  std::vector<int64_t> row_ptr{0};
  std::vector<uint64_t> keys;
  std::vector<float> vals;     // same length as keys, 1.0 for binary features
  std::vector<int32_t> slots;  // slot (feature group) id per nnz
  bool binary = true;          // true if every value is 1 (implicit, or an explicit "k:1")
  int64_t bad_lines = 0;
  std::map<int, SlotStat> info;

  int64_t rows() const { return (int64_t)labels.size(); }
  void append(ParsedBatch&& o);
};

// Parse one line (mutated in place is NOT required; the input is const).
bool parse_line(const char* b, const char* e, const ParseOptions& opt, ParsedBatch* out);
// Parse a buffer of newline separated examples.
ParsedBatch parse_buffer(const char* data, size_t len, const ParseOptions& opt);

// ------------------------------------------------------------------- files
// Whole-file read; ".gz" files are inflated; "hdfs://" paths go through
// `hadoop fs -cat` (reference File::open(DataConfig), src/util/file.cc:50-72).
std::string read_file(const std::string& path, const std::string& hadoop_home = "");
void write_file(const std::string& path, const std::string& data, bool gzip = false);
std::vector<std::string> list_dir(const std::string& dir, const std::string& hadoop_home = "");

// RecordIO framing [u32 magic 0x3ed7230a][u32 len][payload][pad to 4]
// (reference src/util/recordio.h:9,17-77).
constexpr uint32_t kRecordIOMagic = 0x3ed7230a;
std::string recordio_pack(const std::vector<std::string>& records);
std::vector<std::string> recordio_unpack(const std::string& data);

}  // namespace pscore
