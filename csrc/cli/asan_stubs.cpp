// Host-only sanitizer build (make asan): the GPU entry points the CLI links against, as
// stubs that fail loudly.  ASan/UBSan then cover the CPU engine, the loaders, spill I/O,
// the generator, the TCP communicator and the CLI (`--backend cpu`).  Device-side ASan
// (xnack+) is not available on the GPU pool.
#include "locust/dist.hpp"
#include "locust/engine.hpp"
#include "locust/stage.hpp"

namespace locust {

namespace {
[[noreturn]] void no_gpu() { throw Error("this is the host-only sanitizer build: no GPU backend"); }
}  // namespace

struct GpuWordCount::Impl {};
GpuWordCount::GpuWordCount(const JobConfig&, u64, u64) { no_gpu(); }
GpuWordCount::~GpuWordCount() = default;
WordCountResult GpuWordCount::run(const TextInput&) { no_gpu(); }
WordCountResult GpuWordCount::run_source(TextSource&) { no_gpu(); }
char* GpuWordCount::input_buffer() { no_gpu(); }
GpuWordCount::Stats GpuWordCount::stats() const { no_gpu(); }
bool GpuWordCount::partition_map(std::vector<u64>*) { no_gpu(); }
bool GpuWordCount::set_partition_map(const std::vector<u64>&) { no_gpu(); }
std::vector<PackedKey> GpuWordCount::run_map_stage(const TextInput&, WordCountResult*) { no_gpu(); }
WordCountResult GpuWordCount::run_reduce_stage(const PackedKey*, u64) { no_gpu(); }
void copy_device(void*, const void*, u64, bool, void*) { no_gpu(); }
DistResult run_single_process_multi_gpu(const DistConfig&, const TextInput&, LocalComm,
                                        std::vector<DistResult>*) {
  no_gpu();
}
DistResult run_single_process_file(const DistConfig&, const std::string&, LocalComm,
                                   std::vector<DistResult>*) {
  no_gpu();
}
std::vector<WordCountEntry> merge_runs_device(const JobConfig&,
                                              const std::vector<std::vector<KeyCount>>&,
                                              double*) {
  no_gpu();
}
int visible_device_count() { return 0; }
std::vector<int> peer_access_row(int) { return {}; }
LocalComm resolve_local_comm(const DistConfig&, LocalComm) { return LocalComm::kLoopback; }

}  // namespace locust
