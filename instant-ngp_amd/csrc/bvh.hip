// bvh.hip — triangle BVH for the SDF ground truth (TriangleBvh4, src/triangle_bvh.cu).
//
// Host build restated from TriangleBvhWithBranchingFactor<4>::build (triangle_bvh.cu:540-617): each
// node splits its triangle range in two at the median centroid (std::nth_element) along the axis of
// largest centroid variance, twice, into 4 children; ranges of <= n_primitives_per_leaf (8,
// testbed_sdf.cu:1157) triangles become leaves. The triangle array is reordered in place exactly as
// the reference reorders m_sdf.triangles_cpu (same algorithm, same libstdc++ nth_element), and the
// surface-sampling CDF is built over that order afterwards (testbed_sdf.cu:1157-1172).
//
// Device queries restated from triangle_bvh.cu:240-433 with a per-thread 32-entry stack
// (FixedIntStack): closest_triangle with the caller's upper bound (children pushed farthest first,
// pruned at push time; no triangle within the bound -> distance 0), and signed_distance_raystab:
// 32 Fibonacci stab rays with the offset random_val_2d of a default pcg32 advanced by 2 i
// (signed_distance_raystab_kernel, :688-703), positive if any ray escapes MAX_DIST = 10. A stab ray
// only needs to know whether any triangle is hit before MAX_DIST, so its traversal stops at the first
// such hit (same sign as the reference's nearest-hit ray_intersect).
#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <stack>
#include <vector>

#include "profiler.h"
#include "training.h"

namespace ngp {

namespace {
constexpr float MAX_DIST = 10.0f;  // triangle_bvh.cu:40
constexpr int STACK = 32;          // FixedStack<int, 32> (triangle_bvh.cuh:34-55)

struct HostTri {
	float v[9];
	float centroid(int axis) const { return (v[axis] + v[3 + axis] + v[6 + axis]) / 3.0f; }
};

void bbox_of(const HostTri* b, const HostTri* e, BvhNode& n) {
	for (int d = 0; d < 3; ++d) n.lo[d] = n.hi[d] = b->v[d];
	for (const HostTri* t = b; t != e; ++t)
		for (int k = 0; k < 3; ++k)
			for (int d = 0; d < 3; ++d) {
				n.lo[d] = std::min(n.lo[d], t->v[3 * k + d]);
				n.hi[d] = std::max(n.hi[d], t->v[3 * k + d]);
			}
}
}  // namespace

void build_bvh4(float* tris, uint32_t n_triangles, uint32_t n_primitives_per_leaf, std::vector<BvhNode>& nodes) {
	NGP_CHECK(n_triangles >= 4, "bvh: need at least 4 triangles");
	// device traversal entries pack a leaf as (first triangle, count - 1) in 25 + 6 bits (node_entry)
	NGP_CHECK(n_primitives_per_leaf <= 64 && n_triangles < (1u << 25), "bvh: at most 64 triangles per leaf and 2^25 triangles");
	HostTri* T = (HostTri*)tris;
	nodes.clear();
	nodes.emplace_back();
	bbox_of(T, T + n_triangles, nodes[0]);
	struct Build { int node; HostTri* b; HostTri* e; };
	std::stack<Build> st;
	st.push({0, T, T + n_triangles});
	while (!st.empty()) {
		const Build cur = st.top();
		st.pop();
		std::array<Build, 4> ch{};
		ch[0] = cur;
		for (int nc = 1; nc < 4; nc *= 2) {
			for (int i = nc - 1; i >= 0; --i) {
				const Build c = ch[i];
				const float cnt = (float)(c.e - c.b);
				float mean[3] = {0.f, 0.f, 0.f};
				for (HostTri* t = c.b; t != c.e; ++t)
					for (int d = 0; d < 3; ++d) mean[d] += (t->v[d] + t->v[3 + d] + t->v[6 + d]) / 3.0f;
				for (int d = 0; d < 3; ++d) mean[d] /= cnt;
				float var[3] = {0.f, 0.f, 0.f};
				for (HostTri* t = c.b; t != c.e; ++t)
					for (int d = 0; d < 3; ++d) {
						const float df = (t->v[d] + t->v[3 + d] + t->v[6 + d]) / 3.0f - mean[d];
						var[d] += df * df;
					}
				for (int d = 0; d < 3; ++d) var[d] /= cnt;
				const float mx = std::max(std::max(var[0], var[1]), var[2]);
				const int axis = var[0] == mx ? 0 : (var[1] == mx ? 1 : 2);
				HostTri* m = c.b + (c.e - c.b) / 2;
				std::nth_element(c.b, m, c.e, [axis](const HostTri& a, const HostTri& b) { return a.centroid(axis) < b.centroid(axis); });
				ch[2 * i].b = c.b;
				ch[2 * i + 1].e = c.e;
				ch[2 * i].e = ch[2 * i + 1].b = m;
			}
		}
		nodes[cur.node].left = (int32_t)nodes.size();
		for (int i = 0; i < 4; ++i) {
			NGP_CHECK(ch[i].b != ch[i].e, "bvh: empty child");
			ch[i].node = (int)nodes.size();
			nodes.emplace_back();
			BvhNode& n = nodes.back();
			bbox_of(ch[i].b, ch[i].e, n);
			if ((uint32_t)(ch[i].e - ch[i].b) <= n_primitives_per_leaf) {
				n.left = -(int32_t)(ch[i].b - T) - 1;
				n.right = -(int32_t)(ch[i].e - T) - 1;
			} else {
				st.push(ch[i]);
			}
		}
		nodes[cur.node].right = (int32_t)nodes.size();
	}
}

namespace {
int host_node_entry(const BvhNode& n) {  // = node_entry on the device
	return n.left >= 0 ? n.left : -(((-n.left - 1) << 6) + (n.left - n.right - 1)) - 1;
}
// fp16 of x rounded toward -inf (down = true) or +inf: the nearest fp16, stepped one ulp outward if it
// lies on the wrong side of x (overflow goes to -/+inf, still outward)
_Float16 f16_outward(float x, bool down) {
	_Float16 h = (_Float16)x;
	const float back = (float)h;
	if (down ? back > x : back < x) {
		uint16_t b;
		std::memcpy(&b, &h, 2);
		const bool neg = b & 0x8000u;
		if ((b & 0x7fffu) == 0) b = down ? 0x8001u : 0x0001u;                 // +-0 -> the smallest subnormal outward
		else if (down) b = neg ? (uint16_t)(b + 1) : (uint16_t)(b - 1);       // toward -inf
		else b = neg ? (uint16_t)(b - 1) : (uint16_t)(b + 1);                 // toward +inf
		std::memcpy(&h, &b, 2);
	}
	return h;
}
}  // namespace

void bvh_child_blocks(const std::vector<BvhNode>& nodes, std::vector<BvhChildBlock>& blocks) {
	NGP_CHECK(nodes.size() >= 5 && (nodes.size() - 1) % 4 == 0, "bvh: children must come in blocks of 4 after the root");
	blocks.assign((nodes.size() - 1) / 4, BvhChildBlock{});
	for (size_t j = 0; j < blocks.size(); ++j)
		for (int c = 0; c < 4; ++c) {
			const BvhNode& n = nodes[1 + 4 * j + c];
			for (int d = 0; d < 3; ++d) {
				blocks[j].lo[c][d] = f16_outward(n.lo[d], true);
				blocks[j].hi[c][d] = f16_outward(n.hi[d], false);
			}
			blocks[j].entry[c] = host_node_entry(n);
		}
}

uint32_t bvh_depth(const std::vector<BvhNode>& nodes) {
	std::vector<uint32_t> d(nodes.size(), 0);  // children are stored after their parent (build order)
	uint32_t deepest = 0;
	for (size_t i = 0; i < nodes.size(); ++i) {
		if (nodes[i].left < 0) continue;
		deepest = std::max(deepest, d[i] + 1);
		for (int c = 0; c < 4; ++c) d[nodes[i].left + c] = d[i] + 1;
	}
	return deepest;
}

// ---- device -----------------------------------------------------------------------------------
namespace {
struct V { float x, y, z; };
__device__ __forceinline__ V vld(const float* p) { return V{p[0], p[1], p[2]}; }
__device__ __forceinline__ V vsub(V a, V b) { return V{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ V vmul(V a, float s) { return V{a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ float vdot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ V vcross(V a, V b) { return V{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
__device__ __forceinline__ float clamp01(float x) { return fminf(fmaxf(x, 0.0f), 1.0f); }
__device__ __forceinline__ float sgn(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

// Triangle::distance_sq (triangle.cuh:66-85)
__device__ float tri_dist_sq(const float* t, V pos) {
	const V A = vld(t), B = vld(t + 3), C = vld(t + 6);
	const V v21 = vsub(B, A), p1 = vsub(pos, A), v32 = vsub(C, B), p2 = vsub(pos, B), v13 = vsub(A, C), p3 = vsub(pos, C);
	const V nor = vcross(v21, v13);
	if (sgn(vdot(vcross(v21, nor), p1)) + sgn(vdot(vcross(v32, nor), p2)) + sgn(vdot(vcross(v13, nor), p3)) < 2.0f) {
		auto edge = [](V v, V p) {
			const V q = vsub(vmul(v, clamp01(vdot(v, p) / vdot(v, v))), p);
			return vdot(q, q);
		};
		return fminf(fminf(edge(v21, p1), edge(v32, p2)), edge(v13, p3));
	}
	const float d = vdot(nor, p1);
	return d * d / vdot(nor, nor);
}

// Triangle::ray_intersect (triangle.cuh:44-58)
__device__ float tri_ray_t(const float* t, V ro, V rd) {
	const V A = vld(t);
	const V v1v0 = vsub(vld(t + 3), A), v2v0 = vsub(vld(t + 6), A), rov0 = vsub(ro, A);
	const V n = vcross(v1v0, v2v0);
	const V q = vcross(rov0, rd);
	const float d = 1.0f / vdot(rd, n);
	const float u = d * -vdot(q, v2v0);
	const float v = d * vdot(q, v1v0);
	float tt = d * -vdot(n, rov0);
	if (u < 0.0f || u > 1.0f || v < 0.0f || (u + v) > 1.0f || tt < 0.0f) tt = 3.402823466e38f;
	return tt;
}

// BoundingBox::distance_sq (bounding_box.cuh:230-232)
__device__ __forceinline__ float box_dist_sq(const BvhNode& n, V p) {
	const float dx = fmaxf(fmaxf(n.lo[0] - p.x, p.x - n.hi[0]), 0.0f);
	const float dy = fmaxf(fmaxf(n.lo[1] - p.y, p.y - n.hi[1]), 0.0f);
	const float dz = fmaxf(fmaxf(n.lo[2] - p.z, p.z - n.hi[2]), 0.0f);
	return dx * dx + dy * dy + dz * dz;
}

// BoundingBox::ray_intersect (bounding_box.cuh:163-216), entry distance
__device__ float box_ray_t(const BvhNode& n, V o, V d) {
	const float FMAX = 3.402823466e+38f;
	float tmin = (n.lo[0] - o.x) / d.x, tmax = (n.hi[0] - o.x) / d.x;
	if (tmin > tmax) { const float t = tmin; tmin = tmax; tmax = t; }
	float tymin = (n.lo[1] - o.y) / d.y, tymax = (n.hi[1] - o.y) / d.y;
	if (tymin > tymax) { const float t = tymin; tymin = tymax; tymax = t; }
	if (tmin > tymax || tymin > tmax) return FMAX;
	if (tymin > tmin) tmin = tymin;
	if (tymax < tmax) tmax = tymax;
	float tzmin = (n.lo[2] - o.z) / d.z, tzmax = (n.hi[2] - o.z) / d.z;
	if (tzmin > tzmax) { const float t = tzmin; tzmin = tzmax; tzmax = t; }
	if (tmin > tzmax || tzmin > tmax) return FMAX;
	if (tzmin > tmin) tmin = tzmin;
	return tmin;
}

template <typename K> __device__ __forceinline__ void sort4_desc(K* k, int* id) {  // sorting_network<4>, largest first
	auto cs = [&](int a, int b) {
		if (k[a] < k[b]) { const K tk = k[a]; k[a] = k[b]; k[b] = tk; const int ti = id[a]; id[a] = id[b]; id[b] = ti; }
	};
	cs(0, 2); cs(1, 3); cs(0, 1); cs(2, 3); cs(1, 2);
}

// Traversal state. A stack entry names what the traversal needs next without re-reading the node it
// came from: an internal node is pushed as the index of its first child (its 4 children are stored
// consecutively, build_bvh4), a leaf as -(first_triangle * 64 + count - 1) - 1. The per-lane stacks live
// in LDS, slot-major ([slot][thread]: consecutive lanes hit consecutive banks); as a register array a
// divergent stack pointer turns every push and pop into a 32-way select chain.
__device__ __forceinline__ int node_entry(const BvhNode& n) {
	return n.left >= 0 ? n.left : -(((-n.left - 1) << 6) + (n.left - n.right - 1)) - 1;
}
// The 4 children of the internal node whose traversal entry is e (their first node index): one 64-B
// child block (4 x 16-B loads) instead of 4 x 32-B BvhNodes; the fp16 boxes enclose the float ones.
struct Children {
	BvhNode n[4];  // boxes widened to fp16-representable bounds; left = traversal entry (right unused)
};
__device__ __forceinline__ Children load_children(const BvhChildBlock* __restrict__ blocks, int e) {
	const f32x4* q = (const f32x4*)(blocks + ((e - 1) >> 2));
	const f32x4 a = q[0], b = q[1], c = q[2], d = q[3];
	typedef _Float16 h8 __attribute__((ext_vector_type(8)));
	const h8 ha = __builtin_bit_cast(h8, a), hb = __builtin_bit_cast(h8, b), hc = __builtin_bit_cast(h8, c);
	_Float16 h[24];
#pragma unroll
	for (int k = 0; k < 8; ++k) { h[k] = ha[k]; h[8 + k] = hb[k]; h[16 + k] = hc[k]; }
	Children ch;
#pragma unroll
	for (int k = 0; k < 4; ++k) {
#pragma unroll
		for (int t = 0; t < 3; ++t) {
			ch.n[k].lo[t] = (float)h[3 * k + t];
			ch.n[k].hi[t] = (float)h[12 + 3 * k + t];
		}
		ch.n[k].left = __float_as_int(d[k]);
		ch.n[k].right = 0;
	}
	return ch;
}
__device__ __forceinline__ void leaf_range(int e, int& first, int& end) {
	const int v = -e - 1;
	first = v >> 6;
	end = first + (v & 63) + 1;
}

// closest_triangle (triangle_bvh.cu:286-335): squared distance, or -1 if none within max_sq. Same
// arithmetic and pruning as the reference's traversal (children visited nearest first, pruned at push
// time against the best distance so far), with the root's four subtrees searched by the four lanes of a
// group (DIST_G) that share their best distance through LDS: a pruning bound can only be one another
// lane has reached, so the minimum found is the serial search's (the closest triangle is never pruned:
// its box distance is below its own distance).
__device__ float closest_dist_sq(V p, const BvhNode* __restrict__ nodes, const float* __restrict__ tris, float max_sq, int* stk,
                                 int stride, uint32_t* shared_best, int sub) {
	// the nearest accepted child is visited next straight from a register (the reference pushes it last
	// and pops it first: the same order); only its farther siblings go through the LDS stack
	// float boxes here (the fp16 child blocks' looser boxes prune less: 1.32 -> 1.43 ms on the armadillo batch)
	const BvhNode top = nodes[nodes[0].left + sub];  // the root is always internal (build_bvh4 splits it)
	float best = max_sq;
	bool found = false;
	if (box_dist_sq(top, p) > best) return -1.0f;
	int e = node_entry(top);
	int sp = 0;
	while (true) {
		best = fminf(best, __uint_as_float(__hip_atomic_load(shared_best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)));
		if (e < 0) {
			int i, end;
			leaf_range(e, i, end);
			float lb = best;
			for (; i < end; ++i) {
				const float d = tri_dist_sq(tris + 9 * (size_t)i, p);
				if (d <= lb) { lb = d; found = true; }
			}
			if (lb < best) {
				best = lb;
				atomicMin(shared_best, __float_as_uint(lb));  // non-negative floats order as their bits
			}
			if (sp == 0) break;
			e = stk[--sp * stride];
		} else {
			float k[4];
			int id[4];
#pragma unroll
			for (int c = 0; c < 4; ++c) {
				const BvhNode ch = nodes[e + c];
				id[c] = node_entry(ch);
				k[c] = box_dist_sq(ch, p);
			}
			sort4_desc(k, id);
#pragma unroll
			for (int c = 0; c < 3; ++c)
				if (k[c] <= best && sp < STACK) stk[sp++ * stride] = id[c];
			if (k[3] <= best) e = id[3];
			else if (sp == 0) break;
			else e = stk[--sp * stride];
		}
	}
	return found ? best : -1.0f;
}

// fibonacci_dir<32> (random_val.cuh:84-99) + cylindrical_to_dir (:45-54)
__device__ V fib_dir32(uint32_t i, float ox, float oy) {
	const float eps = 1.33f;
	const float golden = 1.6180339887498948482045868343656f;
	float a = (i + eps) / (32 - 1 + 2 * eps) + ox;
	float b = i / golden + oy;
	a = a - floorf(a);
	b = b - floorf(b);
	const float cos_theta = -2.0f * a + 1.0f;
	const float phi = 2.0f * 3.14159265358979323846f * (b - 0.5f);
	const float sin_theta = sqrtf(fmaxf(1.0f - cos_theta * cos_theta, 0.0f));
	float sp, cp;
	sincosf(phi, &sp, &cp);
	return V{sin_theta * cp, sin_theta * sp, cos_theta};
}

__device__ __forceinline__ float pcg_next_float(uint64_t& state, uint64_t inc) {  // tcnn::pcg32::next_float
	const uint64_t old = state;
	state = old * 0x5851f42d4c957f2dULL + inc;
	const uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u), rot = (uint32_t)(old >> 59u);
	const uint32_t u = (xs >> rot) | (xs << ((~rot + 1u) & 31));
	return __uint_as_float((u >> 9) | 0x3f800000u) - 1.0f;
}
__device__ __forceinline__ uint64_t pcg_advanced(uint64_t state, uint64_t inc, uint64_t delta) {  // pcg32::advance
	uint64_t cm = 0x5851f42d4c957f2dULL, cp = inc, am = 1u, ap = 0u;
	while (delta > 0) {
		if (delta & 1) { am *= cm; ap = ap * cm + cp; }
		cp = (cm + 1) * cp;
		cm *= cm;
		delta /= 2;
	}
	return am * state + ap;
}

// Slab test of a stab ray against a child box, widened so that it never rejects a box the reference's
// division-based BoundingBox::ray_intersect (box_ray_t) accepts: the ray's reciprocal direction is
// computed once, each slab distance (lo - o) * (1/d) is within 3 ulp of the quotient (lo - o) / d, and the
// overlap and MAX_DIST tests get a slack of 2^-19 of the magnitudes involved (>= 16 ulp). Accepting extra
// boxes only visits more triangles; the sign is decided by tri_ray_t alone (a triangle hit lies inside
// every box that contains the triangle), so the outcome is the reference's. Rays with a zero direction
// component (0 * inf) take the exact test.
struct StabRay {
	V o, d, id;
	bool exact;
};
__device__ __forceinline__ float stab_box(const BvhNode& n, const StabRay& r) {  // entry distance, or FMAX if rejected
	if (r.exact) return box_ray_t(n, r.o, r.d);
	const float x0 = (n.lo[0] - r.o.x) * r.id.x, x1 = (n.hi[0] - r.o.x) * r.id.x;
	const float y0 = (n.lo[1] - r.o.y) * r.id.y, y1 = (n.hi[1] - r.o.y) * r.id.y;
	const float z0 = (n.lo[2] - r.o.z) * r.id.z, z1 = (n.hi[2] - r.o.z) * r.id.z;
	const float tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1));
	const float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1));
	const float slack = (fabsf(tn) + fabsf(tf)) * 1.9073486e-6f + 1e-30f;  // 2^-19
	return (tn <= tf + slack && tn < MAX_DIST * (1.0f + 1.9073486e-6f)) ? fminf(tn, MAX_DIST * 0.5f) : 3.402823466e+38f;
}

// signed_distance_raystab_kernel (triangle_bvh.cu:688-703) in two launches. Distance: one thread per
// point (closest_triangle under the upper bound). Sign: 32 lanes per point, lane k traces stab ray k —
// the rays of one point traverse similar nodes, so the half-wave stays coherent where one thread would
// run the 32 traversals back to back; the first lane whose ray escapes raises an LDS flag that stops the
// others (the sign only asks whether any ray escapes).
constexpr uint32_t DIST_T = 256, DIST_G = 4;  // 64 points per block, one lane per root subtree
__global__ void __launch_bounds__(DIST_T) k_sdf_distance(uint32_t n, const float* __restrict__ pos, const BvhNode* __restrict__ nodes,
                                                         const float* __restrict__ tris, float* __restrict__ dist, bool upper_bounds) {
	__shared__ int stk[STACK * DIST_T];
	__shared__ uint32_t best[DIST_T / DIST_G];
	__shared__ uint32_t any[DIST_T / DIST_G];
	const uint32_t g = threadIdx.x / DIST_G, sub = threadIdx.x % DIST_G;
	const uint32_t i = blockIdx.x * (DIST_T / DIST_G) + g;
	const float max_d = i < n ? (upper_bounds ? dist[i] : MAX_DIST) : 0.f;
	if (sub == 0) { best[g] = __float_as_uint(max_d * max_d); any[g] = 0u; }
	__syncthreads();
	if (i < n) {
		const float dsq = closest_dist_sq(vld(pos + 3 * (size_t)i), nodes, tris, max_d * max_d, stk + threadIdx.x, DIST_T, &best[g],
		                                  (int)sub);
		if (dsq >= 0.f) atomicOr(&any[g], 1u);
	}
	__syncthreads();
	if (i < n && sub == 0) dist[i] = any[g] ? sqrtf(__uint_as_float(best[g])) : 0.0f;
}

constexpr uint32_t SIGN_T = 256;  // 8 points per block
// per-lane stack: the farther siblings along the current path, at most 3 per internal level, so
// 3 x depth slots never overflow (the armadillo's BVH: 7 internal levels, 21 slots = 21 KB of LDS per
// block). Dynamic LDS sized by the host. (A per-block pool of 32 points' rays drawn by idle lanes was
// measured slower, 4.5 -> 5.1 ms on the armadillo batch: the traversal is bound by the node and
// triangle fetches, not by lanes idling between a ray's end and its point's. A binned-SAH query tree
// cut node visits per ray by ~15 % (33 -> 30) and ran no faster; the reference's median-split tree stays.)
__global__ void __launch_bounds__(SIGN_T) k_sdf_sign(uint32_t n, const float* __restrict__ pos, const BvhNode* __restrict__ nodes,
                                                     const BvhChildBlock* __restrict__ blocks, const float* __restrict__ tris,
                                                     float* __restrict__ dist,
                                                     unsigned long long* __restrict__ stats) {
	__shared__ uint32_t escaped[SIGN_T / 32];
	uint32_t n_inner = 0, n_leaf = 0, n_tri = 0;  // traversal statistics (stats != nullptr: NGP_SDF_STATS)
	extern __shared__ int stk_all[];
	int* stk = stk_all + threadIdx.x;
	const uint32_t g = threadIdx.x / 32, k = threadIdx.x % 32;
	const uint32_t i = blockIdx.x * (SIGN_T / 32) + g;
	if (k == 0) escaped[g] = 0u;
	__syncthreads();
	if (i < n) {
		const V p = vld(pos + 3 * (size_t)i);
		const uint64_t inc = 0xda3e39cb94b95bdbULL;  // default_rng_t advanced by 2 i
		uint64_t st = pcg_advanced(0x853c49e6748fea9bULL, inc, 2ull * i);
		const float ox = pcg_next_float(st, inc), oy = pcg_next_float(st, inc);
		StabRay r;
		r.o = p;
		r.d = fib_dir32(k, ox, oy);
		r.id = V{1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z};
		r.exact = r.d.x == 0.f || r.d.y == 0.f || r.d.z == 0.f;
		// any triangle closer than MAX_DIST along ray k? (stops early once another ray escaped). The node
		// to visit next is kept in a register (`e`): a descent to the nearest accepted child costs no
		// stack round trip; only its farther siblings are pushed.
		int e = nodes[0].left;
		int sp = 0;
		bool hit = false, done = false;
		while (!done) {
			if (__hip_atomic_load(&escaped[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
			if (e < 0) {
				int t, end;
				leaf_range(e, t, end);
				++n_leaf;
				n_tri += end - t;
				for (; t < end && !hit; t += 2) {  // two triangles' loads in flight
					const bool h0 = tri_ray_t(tris + 9 * (size_t)t, p, r.d) < MAX_DIST;
					const bool h1 = t + 1 < end && tri_ray_t(tris + 9 * (size_t)(t + 1), p, r.d) < MAX_DIST;
					hit = h0 || h1;
				}
				if (hit) break;
				if (sp == 0) done = true;
				else e = stk[--sp * SIGN_T];
			} else {
				++n_inner;
				float kk[4];
				int id[4];
				const Children ch = load_children(blocks, e);
#pragma unroll
				for (int c = 0; c < 4; ++c) {
					id[c] = ch.n[c].left;
					kk[c] = stab_box(ch.n[c], r);
				}
				// nearest accepted child next, the others pushed farthest first: only how soon a hit is
				// found depends on the order
				sort4_desc(kk, id);
#pragma unroll
				for (int c = 0; c < 3; ++c)
					if (kk[c] < MAX_DIST) stk[sp++ * SIGN_T] = id[c];
				if (kk[3] < MAX_DIST) e = id[3];
				else if (sp == 0) done = true;
				else e = stk[--sp * SIGN_T];
			}
		}
		if (done) __hip_atomic_store(&escaped[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
	}
	__syncthreads();
	if (i < n && k == 0 && !escaped[g]) dist[i] = -dist[i];
	if (stats && i < n) {
		atomicAdd(&stats[0], (unsigned long long)n_inner);
		atomicAdd(&stats[1], (unsigned long long)n_leaf);
		atomicAdd(&stats[2], (unsigned long long)n_tri);
		atomicAdd(&stats[3], 1ull);
		if (k == 0) {
			atomicAdd(&stats[5], 1ull);
			if (!escaped[g]) atomicAdd(&stats[6], 1ull);
		}
	}
}
}  // namespace

void sdf_signed_distance(const SdfMeshDev& m, uint32_t n, const float* positions, float* distances, bool upper_bounds, hipStream_t s) {
	if (n == 0) return;
	NGP_CHECK(m.qnodes && m.qtris && m.blocks, "sdf: mesh has no BVH");
	{
		ProfScope ps("sdf_distance", s);
		k_sdf_distance<<<div_round_up(n, DIST_T / DIST_G), DIST_T, 0, s>>>(n, positions, m.qnodes, m.qtris, distances, upper_bounds);
		NGP_HIP(hipGetLastError());
	}
	ProfScope ps("sdf_sign", s);
	const size_t lds = (size_t)3 * std::max(m.qdepth, 1u) * SIGN_T * sizeof(int);
	NGP_CHECK(lds <= 64 * 1024, "sdf: BVH too deep for the stab-ray stacks");
	static unsigned long long* stats = nullptr;
	const bool want_stats = getenv("NGP_SDF_STATS") != nullptr;
	if (want_stats && !stats) NGP_HIP(hipMalloc(&stats, 8 * sizeof(unsigned long long)));
	if (want_stats) NGP_HIP(hipMemsetAsync(stats, 0, 8 * sizeof(unsigned long long), s));
	k_sdf_sign<<<div_round_up(n, SIGN_T / 32), SIGN_T, lds, s>>>(n, positions, m.qnodes, m.blocks, m.qtris, distances,
	                                                            want_stats ? stats : nullptr);
	NGP_HIP(hipGetLastError());
	if (want_stats) {  // diagnostics: traversal work per stab ray and per point
		unsigned long long h[8];
		NGP_HIP(hipMemcpyAsync(h, stats, sizeof(h), hipMemcpyDeviceToHost, s));
		NGP_HIP(hipStreamSynchronize(s));
		const double lanes = (double)std::max(h[3], 1ull), groups = (double)std::max(h[5], 1ull);
		fprintf(stderr, "{\"sdf_sign_stats\": {\"points\": %llu, \"inner_per_ray\": %.2f, \"leaf_per_ray\": %.2f, "
		        "\"tris_per_ray\": %.2f, \"inside_frac\": %.4f}}\n",
		        h[5], h[0] / lanes, h[1] / lanes, h[2] / lanes, h[6] / groups);
	}
}

}  // namespace ngp
