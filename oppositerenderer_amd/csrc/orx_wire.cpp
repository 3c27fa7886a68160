// orx_wire.cpp — the reference's client/server framing and the client's merge
// (include/orx_wire.h).  Host code, compiled into liborx.so with
// -ffp-contract=off so the merge rounds exactly like the reference's float
// loops (RenderResultPacket.cpp:104-121, RenderResultPacketReceiver.cpp:166-190).
#include "orx_wire.h"

#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

namespace {

// ---- QDataStream writer / reader (big-endian) ----------------------------
struct Writer {
    uint8_t* p;
    uint64_t n = 0;
    explicit Writer(void* dst) : p((uint8_t*)dst) {}
    void u32(uint32_t v) {
        for (int k = 3; k >= 0; k--) p[n++] = (uint8_t)(v >> (8 * k));
    }
    void u64(uint64_t v) {
        for (int k = 7; k >= 0; k--) p[n++] = (uint8_t)(v >> (8 * k));
    }
    void f64(double v) {
        uint64_t b;
        std::memcpy(&b, &v, 8);
        u64(b);
    }
    void f32(float v) {
        uint32_t b;
        std::memcpy(&b, &v, 4);
        u32(b);
    }
    void raw(const void* s, uint64_t len) {
        if (len) std::memcpy(p + n, s, len);
        n += len;
    }
};

struct Reader {
    const uint8_t* p;
    uint64_t len, n = 0;
    bool ok = true;
    Reader(const void* s, uint64_t l) : p((const uint8_t*)s), len(l) {}
    bool need(uint64_t k) {
        if (!ok || len - n < k) ok = false;
        return ok;
    }
    uint32_t u32() {
        if (!need(4)) return 0;
        uint32_t v = 0;
        for (int k = 0; k < 4; k++) v = (v << 8) | p[n++];
        return v;
    }
    uint64_t u64() {
        if (!need(8)) return 0;
        uint64_t v = 0;
        for (int k = 0; k < 8; k++) v = (v << 8) | p[n++];
        return v;
    }
    double f64() {
        const uint64_t b = u64();
        double v;
        std::memcpy(&v, &b, 8);
        return v;
    }
    float f32() {
        const uint32_t b = u32();
        float v;
        std::memcpy(&v, &b, 4);
        return v;
    }
    const uint8_t* take(uint64_t k) {
        if (!need(k)) return nullptr;
        const uint8_t* s = p + n;
        n += k;
        return s;
    }
};

constexpr uint32_t kNull = 0xffffffffu;

float cam_value(const orx_camera& c, int i) {
    const float v[12] = {c.eye[0], c.eye[1], c.eye[2], c.lookat[0], c.lookat[1], c.lookat[2],
                         c.up[0],  c.up[1],  c.up[2],  c.hfov,      c.vfov,      c.aperture};
    return v[i];
}

uint64_t details_bytes(const orx_wire_request* r) {
    return 12 * 8 + 4 + (r->scene_name ? r->scene_name_len : 0) + 3 * 4 + 8;
}
uint64_t inner_bytes(const orx_wire_request* r) {
    return 8 + 4 + 8ull * r->n_iterations + 4 + 8ull * r->n_radii + 4 + details_bytes(r);
}

// the fields of a request frame after the leading int32 and the inner length
struct RequestFields {
    uint64_t seq = 0;
    uint32_t n_it = 0, n_rad = 0, name_len = 0;
    bool name_null = false;
    const uint8_t* its = nullptr;
    const uint8_t* radii = nullptr;
    const uint8_t* name = nullptr;
    float cam[12] = {};
    uint32_t method = 0, width = 0, height = 0;
    double alpha = 0;
    uint64_t frame = 0;
};

bool parse_request(const void* src, uint64_t len, RequestFields& f) {
    Reader r(src, len);
    const uint32_t framed = r.u32();  // int(inner size + 2*sizeof(int))
    const uint32_t inner_len = r.u32();
    if (!r.ok || inner_len == kNull || framed != inner_len + 8u) return false;
    const uint8_t* inner = r.take(inner_len);
    if (!inner) return false;
    f.frame = r.n;
    Reader in(inner, inner_len);
    f.seq = in.u64();
    f.n_it = in.u32();
    f.its = in.take(8ull * f.n_it);
    f.n_rad = in.u32();
    f.radii = in.take(8ull * f.n_rad);
    const uint32_t dlen = in.u32();
    if (!in.ok || dlen == kNull) return false;
    const uint8_t* det = in.take(dlen);
    if (!det || in.n != inner_len) return false;
    Reader d(det, dlen);
    for (int i = 0; i < 12; i++) f.cam[i] = (float)d.f64();  // operator>>(float) on a double-precision stream
    f.name_len = d.u32();
    f.name_null = f.name_len == kNull;
    if (f.name_null) f.name_len = 0;
    f.name = d.take(f.name_len);
    f.method = d.u32();
    f.width = d.u32();
    f.height = d.u32();
    f.alpha = d.f64();
    return d.ok && d.n == dlen;
}

struct ResultFields {
    uint64_t seq = 0, frame = 0, out_bytes = 0;
    uint32_t n_it = 0;
    const uint8_t* its = nullptr;
    const uint8_t* out = nullptr;
    float render_time = 0, total_time = 0;
};

bool parse_result(const void* src, uint64_t len, ResultFields& f) {
    Reader r(src, len);
    const uint64_t size = r.u64();
    if (!r.ok || size > len - 8) return false;
    f.seq = r.u64();
    f.n_it = r.u32();
    f.its = r.take(8ull * f.n_it);
    f.render_time = r.f32();
    f.total_time = r.f32();
    const uint32_t olen = r.u32();
    if (!r.ok || olen == kNull || (olen & 3u)) return false;
    f.out_bytes = olen;
    f.out = r.take(olen);
    if (!r.ok || r.n != size + 8) return false;
    f.frame = r.n;
    return true;
}

uint64_t be64(const uint8_t* p) {
    uint64_t v = 0;
    for (int k = 0; k < 8; k++) v = (v << 8) | p[k];
    return v;
}

// ---- the client's merge ---------------------------------------------------
struct Packet {
    std::vector<uint64_t> its;  // sorted
    std::vector<float> out;
    uint64_t first() const { return its.front(); }
    uint64_t last() const { return its.back(); }
};

// RenderResultPacket::merge: a absorbs b (RenderResultPacket.cpp:104-121)
void packet_merge(Packet& a, const Packet& b) {
    const int ta = (int)a.its.size(), tb = (int)b.its.size();
    const float scale = 1.f / (float)(ta + tb);
    const float fa = (float)ta, fb = (float)tb;
    float* o = a.out.data();
    const float* in = b.out.data();
    const size_t n = a.out.size();
    for (size_t i = 0; i < n; i++) o[i] = (fa * o[i] + fb * in[i]) * scale;
    a.its.insert(a.its.end(), b.its.begin(), b.its.end());
}

// mergeBufferRunningAverage (RenderResultPacketReceiver.cpp:166-190)
void running_average(const float* in, uint32_t n_in, float* out, uint32_t n_out, size_t n) {
    if (n_out == 0) {
        std::memcpy(out, in, n * sizeof(float));
        return;
    }
    const float total = (float)(n_out + n_in);
    const float ratio = (float)n_in / total;
    for (size_t i = 0; i < n; i++) out[i] = out[i] + (in[i] - out[i]) * ratio;
}

}  // namespace

struct orx_receiver {
    bool ppm = false;
    uint64_t last_sequence = 0;
    uint64_t iteration = 0;
    uint64_t next_expected = 0;
    uint64_t peak_bytes = 0;
    std::vector<float> front;
    bool has_front = false;
    std::vector<Packet> back;  // sorted by first iteration

    void reset() {
        next_expected = 0;
        iteration = 0;
        back.clear();
        peak_bytes = 0;
    }
    uint64_t back_bytes() const {
        uint64_t s = 0;
        for (const Packet& p : back) s += p.out.size() * sizeof(float) + 32;
        return s;
    }
    uint32_t back_iterations() const {
        uint32_t s = 0;
        for (const Packet& p : back) s += (uint32_t)p.its.size();
        return s;
    }
};

extern "C" {

uint64_t orx_wire_request_bytes(const orx_wire_request* r) {
    return r ? 4 + 4 + inner_bytes(r) : 0;
}

orx_status orx_wire_encode_request(const orx_wire_request* r, void* dst, uint64_t cap, uint64_t* written) {
    if (!r || !dst || (r->n_iterations && !r->iteration_numbers) || (r->n_radii && !r->ppm_radii)) return ORX_ERR_INVALID_ARGUMENT;
    const uint64_t total = orx_wire_request_bytes(r);
    const uint64_t inner = inner_bytes(r);
    if (cap < total || inner + 8 > 0x7fffffffull) return ORX_ERR_INVALID_ARGUMENT;
    Writer w(dst);
    w.u32((uint32_t)(inner + 8));  // (int)(array.size() + 2*sizeof(int))
    w.u32((uint32_t)inner);
    w.u64(r->sequence_number);
    w.u32(r->n_iterations);
    for (uint32_t i = 0; i < r->n_iterations; i++) w.u64(r->iteration_numbers[i]);
    w.u32(r->n_radii);
    for (uint32_t i = 0; i < r->n_radii; i++) w.f64(r->ppm_radii[i]);
    w.u32((uint32_t)details_bytes(r));
    for (int i = 0; i < 12; i++) w.f64((double)cam_value(r->camera, i));  // floats on a double-precision stream
    if (r->scene_name) {
        w.u32(r->scene_name_len);
        w.raw(r->scene_name, r->scene_name_len);
    } else {
        w.u32(kNull);
    }
    w.u32(r->render_method);
    w.u32(r->width);
    w.u32(r->height);
    w.f64(r->ppm_alpha);
    if (written) *written = w.n;
    return w.n == total ? ORX_OK : ORX_ERR_STATE;
}

orx_status orx_wire_peek_request(const void* src, uint64_t len, orx_wire_request_info* info) {
    RequestFields f;
    if (!src || !info || !parse_request(src, len, f)) return ORX_ERR_INVALID_ARGUMENT;
    info->frame_bytes = f.frame;
    info->n_iterations = f.n_it;
    info->n_radii = f.n_rad;
    info->scene_name_len = f.name_len;
    info->scene_name_null = f.name_null ? 1 : 0;
    return ORX_OK;
}

orx_status orx_wire_decode_request(const void* src, uint64_t len, orx_wire_request* out, uint64_t* iteration_numbers,
                                   double* ppm_radii, char* scene_name) {
    RequestFields f;
    if (!src || !out || !parse_request(src, len, f)) return ORX_ERR_INVALID_ARGUMENT;
    if ((f.n_it && !iteration_numbers) || (f.n_rad && !ppm_radii) || (f.name_len && !scene_name))
        return ORX_ERR_INVALID_ARGUMENT;
    for (uint32_t i = 0; i < f.n_it; i++) iteration_numbers[i] = be64(f.its + 8ull * i);
    for (uint32_t i = 0; i < f.n_rad; i++) {
        const uint64_t b = be64(f.radii + 8ull * i);
        std::memcpy(&ppm_radii[i], &b, 8);
    }
    if (f.name_len) std::memcpy(scene_name, f.name, f.name_len);
    std::memset(out, 0, sizeof *out);
    out->sequence_number = f.seq;
    out->n_iterations = f.n_it;
    out->n_radii = f.n_rad;
    out->iteration_numbers = iteration_numbers;
    out->ppm_radii = ppm_radii;
    float* c[12] = {&out->camera.eye[0],    &out->camera.eye[1],    &out->camera.eye[2], &out->camera.lookat[0],
                    &out->camera.lookat[1], &out->camera.lookat[2], &out->camera.up[0],  &out->camera.up[1],
                    &out->camera.up[2],     &out->camera.hfov,      &out->camera.vfov,   &out->camera.aperture};
    for (int i = 0; i < 12; i++) *c[i] = f.cam[i];
    out->scene_name = f.name_null ? nullptr : (scene_name ? scene_name : "");
    out->scene_name_len = f.name_len;
    out->render_method = f.method;
    out->width = f.width;
    out->height = f.height;
    out->ppm_alpha = f.alpha;
    return ORX_OK;
}

uint64_t orx_wire_result_bytes(const orx_wire_result* p) {
    return p ? 8 + 8 + 4 + 8ull * p->n_iterations + 4 + 4 + 4 + p->output_bytes : 0;
}

orx_status orx_wire_encode_result(const orx_wire_result* p, void* dst, uint64_t cap, uint64_t* written) {
    if (!p || !dst || (p->n_iterations && !p->iteration_numbers) || (p->output_bytes && !p->output) ||
        p->output_bytes >= kNull)
        return ORX_ERR_INVALID_ARGUMENT;
    const uint64_t total = orx_wire_result_bytes(p);
    if (cap < total) return ORX_ERR_INVALID_ARGUMENT;
    std::vector<uint64_t> its(p->iteration_numbers, p->iteration_numbers + p->n_iterations);
    std::sort(its.begin(), its.end());  // qSort(iterationNumbersInPacket)
    // RenderResultPacket.cpp:134-139: output + its length field, the vector, the sequence number, two floats
    const uint64_t size = (p->output_bytes + 4) + (8ull * p->n_iterations + 4) + 8 + 2 * 4;
    Writer w(dst);
    w.u64(size);
    w.u64(p->sequence_number);
    w.u32(p->n_iterations);
    for (uint64_t v : its) w.u64(v);
    w.f32(p->render_time_seconds);  // SinglePrecision socket stream
    w.f32(p->total_time_seconds);
    w.u32((uint32_t)p->output_bytes);
    w.raw(p->output, p->output_bytes);
    if (written) *written = w.n;
    return w.n == total ? ORX_OK : ORX_ERR_STATE;
}

orx_status orx_wire_peek_result(const void* src, uint64_t len, orx_wire_result_info* info) {
    ResultFields f;
    if (!src || !info || !parse_result(src, len, f)) return ORX_ERR_INVALID_ARGUMENT;
    info->frame_bytes = f.frame;
    info->n_iterations = f.n_it;
    info->reserved = 0;
    info->output_bytes = f.out_bytes;
    return ORX_OK;
}

orx_status orx_wire_decode_result(const void* src, uint64_t len, orx_wire_result* out, uint64_t* iteration_numbers,
                                  float* output) {
    ResultFields f;
    if (!src || !out || !parse_result(src, len, f)) return ORX_ERR_INVALID_ARGUMENT;
    if ((f.n_it && !iteration_numbers) || (f.out_bytes && !output)) return ORX_ERR_INVALID_ARGUMENT;
    for (uint32_t i = 0; i < f.n_it; i++) iteration_numbers[i] = be64(f.its + 8ull * i);
    if (f.out_bytes) std::memcpy(output, f.out, f.out_bytes);
    std::memset(out, 0, sizeof *out);
    out->sequence_number = f.seq;
    out->n_iterations = f.n_it;
    out->iteration_numbers = iteration_numbers;
    out->render_time_seconds = f.render_time;
    out->total_time_seconds = f.total_time;
    out->output = output;
    out->output_bytes = f.out_bytes;
    return ORX_OK;
}

orx_status orx_receiver_create(int32_t method, orx_receiver** out) {
    if (!out) return ORX_ERR_INVALID_ARGUMENT;
    orx_receiver* r = new (std::nothrow) orx_receiver();
    if (!r) return ORX_ERR_OUT_OF_MEMORY;
    r->ppm = method == ORX_METHOD_PROGRESSIVE_PHOTON_MAPPING;
    *out = r;
    return ORX_OK;
}

void orx_receiver_destroy(orx_receiver* r) { delete r; }

orx_status orx_receiver_push(orx_receiver* r, const orx_wire_result* packet, uint64_t current_sequence,
                             int32_t* accepted) {
    if (accepted) *accepted = 0;
    if (!r || !packet || !packet->n_iterations || !packet->iteration_numbers || (packet->output_bytes & 3u) ||
        (packet->output_bytes && !packet->output))
        return ORX_ERR_INVALID_ARGUMENT;
    // onRenderResultPacketReceived (RenderResultPacketReceiver.cpp:30-58)
    if (packet->sequence_number != current_sequence) return ORX_OK;
    if (packet->sequence_number > r->last_sequence) {
        r->reset();
        r->last_sequence = packet->sequence_number;
    }
    const size_t n = packet->output_bytes / sizeof(float);
    if (r->has_front && r->front.size() != n && (r->iteration || r->next_expected || !r->back.empty()))
        return ORX_ERR_INVALID_ARGUMENT;  // a different frame size inside one sequence
    if (r->front.size() != n) r->front.assign(n, 0.f);
    Packet p;
    p.its.assign(packet->iteration_numbers, packet->iteration_numbers + packet->n_iterations);
    std::sort(p.its.begin(), p.its.end());
    if (r->ppm) {
        // mergeRenderResultPacketPhotonMapping (:66-148)
        p.out.assign(packet->output, packet->output + n);
        auto pos = std::upper_bound(r->back.begin(), r->back.end(), p,
                                    [](const Packet& a, const Packet& b) { return a.first() < b.first(); });
        r->back.insert(pos, std::move(p));
        for (bool merged = true; merged;) {  // combine any two sequential back buffers
            merged = false;
            for (size_t k = 0; k + 1 < r->back.size(); k++) {
                if (r->back[k].last() + 1 == r->back[k + 1].first()) {
                    packet_merge(r->back[k], r->back[k + 1]);
                    r->back.erase(r->back.begin() + (ptrdiff_t)(k + 1));
                    merged = true;
                    break;
                }
            }
        }
        if (r->back.front().first() == r->next_expected) {
            const Packet& b = r->back.front();
            running_average(b.out.data(), (uint32_t)b.its.size(), r->front.data(), (uint32_t)r->next_expected, n);
            r->next_expected = b.last() + 1;
            r->back.erase(r->back.begin());
        }
        r->peak_bytes = std::max(r->peak_bytes, r->back_bytes());
        r->iteration = r->next_expected > 0 ? r->next_expected - 1 : 0;
    } else {
        // mergeRenderResultPathTracing (:153-160)
        running_average(packet->output, packet->n_iterations, r->front.data(), (uint32_t)r->iteration, n);
        r->iteration += packet->n_iterations;
    }
    r->has_front = true;
    if (accepted) *accepted = 1;
    return ORX_OK;
}

orx_status orx_receiver_push_encoded(orx_receiver* r, const void* src, uint64_t len, uint64_t current_sequence,
                                     int32_t* accepted) {
    orx_wire_result_info info;
    orx_status s = orx_wire_peek_result(src, len, &info);
    if (s != ORX_OK) return s;
    std::vector<uint64_t> its(info.n_iterations);
    std::vector<float> out(info.output_bytes / sizeof(float));
    orx_wire_result p;
    s = orx_wire_decode_result(src, len, &p, its.data(), out.data());
    if (s != ORX_OK) return s;
    return orx_receiver_push(r, &p, current_sequence, accepted);
}

const float* orx_receiver_front(const orx_receiver* r, uint64_t* n_floats) {
    if (n_floats) *n_floats = r && r->has_front ? r->front.size() : 0;
    return r && r->has_front ? r->front.data() : nullptr;
}
uint64_t orx_receiver_iteration_number(const orx_receiver* r) { return r ? r->iteration : 0; }
uint64_t orx_receiver_next_expected(const orx_receiver* r) { return r ? r->next_expected : 0; }
uint32_t orx_receiver_backbuffer_iterations(const orx_receiver* r) { return r ? r->back_iterations() : 0; }
uint64_t orx_receiver_backbuffer_bytes(const orx_receiver* r) { return r ? r->back_bytes() : 0; }
uint64_t orx_receiver_peak_backbuffer_bytes(const orx_receiver* r) { return r ? r->peak_bytes : 0; }
int32_t orx_receiver_backbuffer_is_not_filled(const orx_receiver* r, uint64_t current_sequence) {
    if (!r) return 0;
    return (r->last_sequence != current_sequence || r->back_iterations() < 100) ? 1 : 0;
}

}  // extern "C"
