// GeoTIFF tile reader for the DEM mosaic (map_generation/data_manager.py:11-17 reads the DEM
// through rasterio over data/raw/nagasaki_geotiff/mergeLL.vrt: 2 035 Float32 tiles of 225 x 150
// with one <ComplexSource> each).  The VRT is parsed by the host Python (vrt.py); this file
// reads the tiles' pixels, in parallel, straight into the caller's staging buffer (page-locked
// when the caller allocates it so), from which uam_dem_mosaic places them on the device.
//
// Supported: classic little-endian TIFF, one Float32 sample per pixel (SampleFormat 3,
// BitsPerSample 32), strips, no predictor, compression none (1) or deflate (8 / 32946) --
// what the reference tiles and geotiff.write_geotiff use.  Anything else fails loudly with the
// tile's path.
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <exception>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/uampath.h"
#include "polyproc.h"  // uam_fail_: the thread-local uam_last_error() text

namespace {

enum : uint16_t {
    T_WIDTH = 256, T_LENGTH = 257, T_BPS = 258, T_COMPRESSION = 259, T_STRIP_OFFSETS = 273,
    T_SPP = 277, T_ROWS_PER_STRIP = 278, T_STRIP_BYTES = 279, T_PREDICTOR = 317,
    T_SAMPLE_FORMAT = 339
};

struct Tags {
    uint32_t width = 0, length = 0, bps = 32, compression = 1, spp = 1, rps = 0, predictor = 1,
             sformat = 3;
    std::vector<uint32_t> offsets, counts;
};

bool rd16(const std::vector<uint8_t>& b, size_t o, uint16_t* v) {
    if (o + 2 > b.size()) return false;
    std::memcpy(v, b.data() + o, 2);
    return true;
}
bool rd32(const std::vector<uint8_t>& b, size_t o, uint32_t* v) {
    if (o + 4 > b.size()) return false;
    std::memcpy(v, b.data() + o, 4);
    return true;
}

// the IFD entry's values (SHORT or LONG) as uint32
bool values(const std::vector<uint8_t>& b, uint16_t typ, uint32_t count, size_t entry,
            std::vector<uint32_t>* out) {
    const size_t sz = typ == 3 ? 2 : typ == 4 ? 4 : 0;
    if (!sz) return false;
    size_t off = entry + 8;
    // a malformed count (up to 2^32) must fail here, not in resize: the values have to lie
    // inside the file
    if ((uint64_t)sz * count > (uint64_t)b.size()) return false;
    if ((uint64_t)sz * count > 4) {
        uint32_t o;
        if (!rd32(b, off, &o)) return false;
        off = o;
    }
    if ((uint64_t)off + (uint64_t)sz * count > (uint64_t)b.size()) return false;
    out->resize(count);
    for (uint32_t i = 0; i < count; ++i) {
        if (sz == 2) {
            uint16_t v;
            if (!rd16(b, off + 2 * (size_t)i, &v)) return false;
            (*out)[i] = v;
        } else if (!rd32(b, off + 4 * (size_t)i, &(*out)[i])) {
            return false;
        }
    }
    return true;
}

const char* parse(const std::vector<uint8_t>& b, Tags* t) {
    if (b.size() < 8 || std::memcmp(b.data(), "II*\0", 4) != 0)
        return "only little-endian classic TIFF is supported";
    uint32_t ifd;
    uint16_t n;
    if (!rd32(b, 4, &ifd) || !rd16(b, ifd, &n)) return "truncated TIFF header";
    for (uint16_t i = 0; i < n; ++i) {
        const size_t e = ifd + 2 + 12 * (size_t)i;
        uint16_t tag, typ;
        uint32_t count;
        if (!rd16(b, e, &tag) || !rd16(b, e + 2, &typ) || !rd32(b, e + 4, &count))
            return "truncated IFD";
        std::vector<uint32_t> v;
        switch (tag) {
            case T_WIDTH: case T_LENGTH: case T_BPS: case T_COMPRESSION: case T_SPP:
            case T_ROWS_PER_STRIP: case T_PREDICTOR: case T_SAMPLE_FORMAT:
                if (!values(b, typ, count, e, &v) || v.empty()) return "bad tag value";
                if (tag == T_WIDTH) t->width = v[0];
                if (tag == T_LENGTH) t->length = v[0];
                if (tag == T_BPS) t->bps = v[0];
                if (tag == T_COMPRESSION) t->compression = v[0];
                if (tag == T_SPP) t->spp = v[0];
                if (tag == T_ROWS_PER_STRIP) t->rps = v[0];
                if (tag == T_PREDICTOR) t->predictor = v[0];
                if (tag == T_SAMPLE_FORMAT) t->sformat = v[0];
                break;
            case T_STRIP_OFFSETS:
                if (!values(b, typ, count, e, &t->offsets)) return "bad StripOffsets";
                break;
            case T_STRIP_BYTES:
                if (!values(b, typ, count, e, &t->counts)) return "bad StripByteCounts";
                break;
            default:
                break;
        }
    }
    if (t->bps != 32 || t->sformat != 3) return "only Float32 samples are supported";
    if (t->spp != 1) return "only single-band rasters are supported";
    if (t->predictor != 1) return "TIFF predictors are not supported";
    if (t->compression != 1 && t->compression != 8 && t->compression != 32946)
        return "TIFF compression is not supported (none or deflate only)";
    if (t->offsets.empty() || t->offsets.size() != t->counts.size()) return "no strips";
    if (t->rps == 0) t->rps = t->length;
    return nullptr;
}

// one tile into dst [th][tw]
const char* read_tile(const char* path, int32_t th, int32_t tw, float* dst,
                      std::vector<uint8_t>* buf) {
    FILE* f = std::fopen(path, "rb");
    if (!f) return "cannot open";
    std::fseek(f, 0, SEEK_END);
    const long sz = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    if (sz <= 0) {
        std::fclose(f);
        return "empty file";
    }
    buf->resize((size_t)sz);
    const size_t got = std::fread(buf->data(), 1, (size_t)sz, f);
    std::fclose(f);
    if (got != (size_t)sz) return "short read";
    Tags t;
    const char* err = parse(*buf, &t);
    if (err) return err;
    if ((int64_t)t.width != tw || (int64_t)t.length != th)
        return "tile size differs from the mosaic's SrcRect";
    const size_t row = (size_t)tw * 4;
    // the strips must cover every row: dst is a reused ring buffer, so an uncovered row would
    // silently keep a previous chunk's pixels
    if ((uint64_t)t.offsets.size() * t.rps < (uint64_t)th) return "strips do not cover the tile";
    for (size_t s = 0; s < t.offsets.size(); ++s) {
        const uint64_t r0 = (uint64_t)s * t.rps;
        if (r0 >= (uint64_t)th) break;
        const uint64_t rows = std::min<uint64_t>(t.rps, (uint64_t)th - r0);
        const uint64_t o = t.offsets[s], n = t.counts[s];
        if (o + n > buf->size()) return "strip outside the file";
        uint8_t* out = reinterpret_cast<uint8_t*>(dst) + r0 * row;
        if (t.compression == 1) {
            if (n < rows * row) return "short strip";
            std::memcpy(out, buf->data() + o, rows * row);
        } else {
            uLongf dl = (uLongf)(rows * row);
            if (uncompress(out, &dl, buf->data() + o, (uLong)n) != Z_OK || dl != rows * row)
                return "deflate strip does not decode to its rows";
        }
    }
    return nullptr;
}

// A pool of reader threads over one call: read(i0, i1, dst) reads tiles [i0, i1) into
// dst [i1 - i0][th][tw] with every thread of the pool, and returns once all are in.
class TileReaderPool {
   public:
    TileReaderPool(const char* const* paths, int32_t th, int32_t tw, int nt)
        : paths_(paths), th_(th), tw_(tw) {
        for (int k = 1; k < nt; ++k) pool_.emplace_back([this] { loop(); });
    }
    ~TileReaderPool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            quit_ = true;
        }
        cv_.notify_all();
        for (auto& t : pool_) t.join();
    }
    // false on a failed tile (first one in tile order: error())
    bool read(int32_t i0, int32_t i1, float* dst) {
        {
            std::lock_guard<std::mutex> g(mu_);
            i0_ = i0, i1_ = i1, dst_ = dst;
            next_.store(i0);
            busy_ = (int)pool_.size();
            ++gen_;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [this] { return busy_ == 0; });
        return err_tile_ < 0;
    }
    const std::string& error() const { return err_; }

   private:
    void work() {
        std::vector<uint8_t>& buf = tl_buf();
        for (;;) {
            const int32_t i = next_.fetch_add(1);
            if (i >= i1_) return;
            // no exception may leave a pool thread (std::terminate would end the process):
            // allocation failures become the tile's error
            const char* e;
            try {
                e = read_tile(paths_[i], th_, tw_, dst_ + (size_t)(i - i0_) * th_ * tw_, &buf);
            } catch (const std::exception&) {
                e = "out of memory reading the tile";
            }
            if (e) {
                std::lock_guard<std::mutex> g(emu_);
                if (err_tile_ < 0 || i < err_tile_) {
                    err_tile_ = i;
                    err_ = std::string(paths_[i]) + ": " + e;
                }
            }
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return quit_ || gen_ != seen; });
                if (quit_) return;
                seen = gen_;
            }
            work();
            std::lock_guard<std::mutex> g(mu_);
            if (--busy_ == 0) done_cv_.notify_all();
        }
    }
    static std::vector<uint8_t>& tl_buf() {
        thread_local std::vector<uint8_t> b;
        return b;
    }
    const char* const* paths_;
    int32_t th_, tw_;
    std::vector<std::thread> pool_;
    std::mutex mu_, emu_;
    std::condition_variable cv_, done_cv_;
    bool quit_ = false;
    uint64_t gen_ = 0;
    int busy_ = 0;
    int32_t i0_ = 0, i1_ = 0;
    float* dst_ = nullptr;
    std::atomic<int32_t> next_{0};
    int32_t err_tile_ = -1;
    std::string err_;
};

int pool_threads(int32_t n_threads, int32_t n_tiles) {
    // default: the machine's threads up to 16 (a GPU box's CPU share)
    int nt = n_threads > 0 ? n_threads : std::min(16, (int)std::thread::hardware_concurrency());
    return std::max(1, std::min({nt, 64, (int)n_tiles}));
}

}  // namespace

extern "C" int uam_read_tiles(const char* const* paths, int32_t n_tiles, int32_t th, int32_t tw,
                              float* dst, int32_t n_threads) {
    if (n_tiles < 0 || th <= 0 || tw <= 0 || (n_tiles > 0 && (!paths || !dst)))
        return uam_fail_(UAM_E_INVALID, "uam_read_tiles: bad arguments");
    if (n_tiles == 0) return UAM_OK;
    TileReaderPool pool(paths, th, tw, pool_threads(n_threads, n_tiles));
    if (!pool.read(0, n_tiles, dst)) return uam_fail_(UAM_E_INVALID, "%s", pool.error().c_str());
    return UAM_OK;
}

// uam_load_tiles (uampath.hip) streams chunks through its page-locked ring with this
int tiles_stream(const char* const* paths, int32_t n_tiles, int32_t th, int32_t tw,
                 int32_t n_threads, int32_t per_chunk,
                 const std::function<float*(int32_t chunk)>& slot,
                 const std::function<int(int32_t chunk, int32_t i0, int32_t i1)>& filled) {
    TileReaderPool pool(paths, th, tw, pool_threads(n_threads, n_tiles));
    for (int32_t c = 0, i0 = 0; i0 < n_tiles; ++c, i0 += per_chunk) {
        const int32_t i1 = std::min(n_tiles, i0 + per_chunk);
        float* dst = slot(c);
        if (!dst) return UAM_E_HIP;
        if (!pool.read(i0, i1, dst)) return uam_fail_(UAM_E_INVALID, "%s", pool.error().c_str());
        const int st = filled(c, i0, i1);
        if (st) return st;
    }
    return UAM_OK;
}
