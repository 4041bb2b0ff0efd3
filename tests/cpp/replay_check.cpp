// replay_check.cpp -- CPU checks of include/freeimpala_amd/replay.hpp and flags.hpp against
// the reference semantics they restate (data_structures.h:43-481, cmd/freeimpala/main.cpp).
// Prints "OK replay" and exits 0 when every check holds.
#include <cstdio>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <thread>
#include <vector>

#include "freeimpala_amd/device_learner.hpp"
#include "freeimpala_amd/flags.hpp"
#include "freeimpala_amd/learner.hpp"
#include "freeimpala_amd/replay.hpp"

using namespace freeimpala_amd;

#define CHECK(c)                                                                  \
    do {                                                                          \
        if (!(c)) {                                                               \
            std::fprintf(stderr, "CHECK failed at line %d: %s\n", __LINE__, #c);  \
            return 1;                                                             \
        }                                                                         \
    } while (0)

static std::vector<char> entry(size_t bytes, char tag) {
    std::vector<char> e(bytes);
    for (size_t i = 0; i < bytes; ++i) e[i] = (char)(tag + i % 7);
    return e;
}

static int buffer_checks() {
    // FIFO, capacity, try_write when full, readBatch copies (data_structures.h:219-300)
    SharedBuffer sb(2, 3);  // 2 elements = 2 KiB entries, capacity 3
    CHECK(sb.entryBytes() == 2048 && sb.getFilledCount() == 0);
    CHECK(sb.write(entry(2048, 1)) && sb.write(entry(1000, 2)) && sb.try_write(entry(2048, 3)));
    CHECK(!sb.try_write(entry(16, 4)));  // full
    CHECK(!SharedBuffer(1, 2).write(entry(1025, 0)));  // larger than an entry
    auto b = sb.readBatch(2);
    CHECK(b.size() == 2 && b[0] == entry(2048, 1) && b[1].size() == 2048);
    CHECK(std::memcmp(b[1].data(), entry(1000, 2).data(), 1000) == 0);
    CHECK(sb.getFilledCount() == 1);
    // readBatchInto: same FIFO order, first `stride` bytes of each entry
    CHECK(sb.write(entry(2048, 5)));
    std::vector<char> dst(2 * 1024);
    CHECK(sb.readBatchInto(2, dst.data(), 1024));
    CHECK(std::memcmp(dst.data(), entry(2048, 3).data(), 1024) == 0);
    CHECK(std::memcmp(dst.data() + 1024, entry(2048, 5).data(), 1024) == 0);
    CHECK(!sb.readBatchInto(1, dst.data(), 4096));  // stride beyond an entry
    // a blocked reader wakes on setDraining and gets {} with fewer than M entries (:273-280)
    CHECK(sb.write(entry(2048, 6)));
    std::vector<std::vector<char>> got{{'x'}};
    bool into = true;
    std::thread r([&] { got = sb.readBatch(2); });
    std::thread r2([&] {
        std::vector<char> d(4096);
        into = sb.readBatchInto(2, d.data(), 2048);
    });
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    sb.setDraining();
    r.join();
    r2.join();
    CHECK(got.empty() && !into && sb.getFilledCount() == 1);
    // draining with a full batch still hands it out
    SharedBuffer sb2(1, 4);
    CHECK(sb2.write(entry(1024, 7)) && sb2.write(entry(1024, 8)));
    sb2.setDraining();
    CHECK(sb2.readBatch(2).size() == 2 && sb2.readBatch(1).empty());
    // a blocked writer proceeds when a reader frees a slot
    SharedBuffer sb3(1, 1);
    CHECK(sb3.write(entry(1024, 9)));
    bool wrote = false;
    std::thread w([&] { wrote = sb3.write(entry(1024, 10)); });
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    CHECK(!wrote);
    CHECK(sb3.readBatch(1)[0] == entry(1024, 9));
    w.join();
    CHECK(wrote && sb3.readBatch(1)[0] == entry(1024, 10));
    // a writer blocked on a full buffer is released by setDraining with false (the learner's
    // worker drains its buffer when it fails, so actors do not hang on it); a draining buffer
    // with space still takes entries
    SharedBuffer sb4(1, 1);
    CHECK(sb4.write(entry(1024, 11)));
    bool wrote4 = true;
    std::thread w4([&] { wrote4 = sb4.write(entry(1024, 12)); });
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    sb4.setDraining();
    w4.join();
    CHECK(!wrote4 && sb4.getFilledCount() == 1);
    CHECK(sb4.readBatch(1)[0] == entry(1024, 11) && sb4.write(entry(1024, 13)) && sb4.getFilledCount() == 1);
    return 0;
}

static int model_checks(const std::string& dir) {
    namespace fs = std::filesystem;
    fs::remove_all(dir);
    // file format: u64 version || blob (data_structures.h:62-113)
    ModelManager mm(2, 64, dir);
    std::vector<char> blob(64);
    for (int i = 0; i < 64; ++i) blob[i] = (char)(3 * i);
    auto m = mm.getModel(1)->createCopy();
    m->update(blob, 17);
    mm.updateModel(1, m);
    CHECK(mm.getLatestVersion(1) == 17 && mm.getModel(1)->getData() == blob);
    m->update(std::vector<char>(63), 99);  // wrong size: ignored (:143)
    CHECK(m->getVersion() == 17);
    CHECK(mm.waitForModelUpdate(1, 16, 1) && !mm.waitForModelUpdate(1, 17, 1));
    const std::string v = mm.saveModel(1, 5);
    CHECK(v == dir + "/model_1_5.bin" && fs::file_size(v) == 8 + 64);
    std::ifstream f(v, std::ios::binary);
    uint64_t ver = 0;
    std::vector<char> back(64);
    f.read((char*)&ver, 8);
    f.read(back.data(), 64);
    CHECK(ver == 17 && back == blob);
    CHECK(fs::exists(dir + "/model_1_latest.bin"));
    // loadModels: _latest when present, else the highest numbered checkpoint (:337-385)
    ModelManager mm2(2, 64, dir + "/other");
    mm2.loadModels(dir);
    CHECK(mm2.getLatestVersion(1) == 17 && mm2.getModel(1)->getData() == blob);
    fs::remove(dir + "/model_1_latest.bin");
    m->update(std::vector<char>(64, 1), 30);
    mm.updateModel(1, m);
    mm.saveModel(1, 12);
    fs::remove(dir + "/model_1_latest.bin");
    { std::ofstream junk(dir + "/model_1_x.bin"); }
    ModelManager mm3(2, 64, dir + "/third");
    mm3.loadModels(dir);
    CHECK(mm3.getLatestVersion(1) == 30 && mm3.getModel(1)->getFilePath() == dir + "/model_1_12.bin");
    CHECK(detail::state_path_for(dir + "/model_1_12.bin") == dir + "/model_1_12.state");
    // saveModel(p, 0) numbers checkpoints from the counter: after loading model_1_12 it is 13
    CHECK(mm3.saveModel(1) == dir + "/third/model_1_13.bin");
    return 0;
}

static int flag_checks() {
    // the reference's flags + the learner flags, strict
    auto make = [] {
        ArgumentParser p("t");
        p.add_argument("-p", "--players").default_value(2).scan<'i', int>();
        p.add_argument("-M", "--batch-size").default_value(5).scan<'i', int>();
        p.add_argument("-S", "--entry-size").default_value(100).scan<'i', int>();
        p.add_argument("--seed").default_value(7u).scan<'u', unsigned>();
        p.add_argument("--log-level").default_value(std::string("info")).choices("info", "off");
        add_learner_arguments(p);
        return p;
    };
    {
        auto p = make();
        const char* argv[] = {"t", "-p", "1", "--batch-size=32", "-S", "101", "--seq-length", "100",
                              "--lr", "1e-3", "--devices", "0,3", "--learner-seed", "9"};
        p.parse_args(14, argv);
        const LearnerConfig c = LearnerConfig::from_parser(p);
        CHECK(c.players == 1 && c.batch_size == 32 && c.entry_size == 101 && c.seq_length == 100);
        CHECK(c.devices.size() == 2 && c.devices[1] == 3 && c.seed == 9 && std::fabs(c.lr - 1e-3f) < 1e-9f);
        CHECK(p.get<unsigned>("--seed") == 7u && !p.is_used("--seed") && p.is_used("--lr"));
    }
    auto throws = [&](std::vector<const char*> a) {
        auto p = make();
        try {
            p.parse_args((int)a.size(), a.data());
            LearnerConfig::from_parser(p);
        } catch (const std::exception&) {
            return true;
        }
        return false;
    };
    CHECK(throws({"t", "--no-such-flag", "1"}));
    CHECK(throws({"t", "-p", "2x"}));
    CHECK(throws({"t", "--seed", "-3"}));
    CHECK(throws({"t", "--log-level", "loud"}));
    CHECK(throws({"t", "--learner-arch", "resnet"}));
    CHECK(throws({"t", "--lr", "fast"}));
    CHECK(throws({"t", "--batch-size"}));
    CHECK(!throws({"t", "--seq-length", "200", "-S", "10"}));  // the Learner lowers T itself
    return 0;
}

int main(int argc, char** argv) {
    const std::string dir = argc > 1 ? argv[1] : "/tmp/fi_replay_check";
    if (buffer_checks() || model_checks(dir) || flag_checks()) return 1;
    std::printf("OK replay\n");
    return 0;
}
