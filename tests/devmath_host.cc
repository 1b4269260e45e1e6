// Host build of the device numerics (libyafaray_amd/csrc/devmath.h) with extern "C" wrappers, so
// tests/test_devmath.py can pin the exact code the kernels run against the reference's golden
// vectors (tests/golden/prims.npz).  Compiled with g++ -ffp-contract=off at test time.
#include "../libyafaray_amd/csrc/devmath.h"
using namespace yafamd;
extern "C" {
void dm_ri(int which, const uint32_t *b, const uint32_t *r, float *o, int n)
{
	for(int i = 0; i < n; ++i) o[i] = which == 0 ? riVdC(b[i], r[i]) : which == 1 ? riS(b[i], r[i]) : riLp(b[i], r[i]);
}
int dm_udiv_check(uint32_t d, const uint32_t *n, int cnt)
{
	const UDiv q = udivMake(d);
	for(int i = 0; i < cnt; ++i) if(udiv(n[i], q) != n[i] / d) return i;
	return -1;
}
void dm_fnv(const uint32_t *in, uint32_t *o, int n) { for(int i = 0; i < n; ++i) o[i] = fnv32(in[i]); }
void dm_lds(const uint8_t *perm, uint32_t base, double f, const uint32_t *idx, double *o, int n)
{
	const UDiv dv = udivMake(base);
	for(int i = 0; i < n; ++i) o[i] = lowDiscrepancy(perm, base, dv, f, idx[i]);
}
void dm_halton_first(uint32_t base, const uint32_t *start, float *o, int n)
{
	for(int i = 0; i < n; ++i) o[i] = haltonFirst(base, 1.0 / (double)base, start[i]);
}
void dm_sin(const float *x, float *o, int n) { for(int i = 0; i < n; ++i) o[i] = fsin(x[i]); }
void dm_cos(const float *x, float *o, int n) { for(int i = 0; i < n; ++i) o[i] = fcos(x[i]); }
void dm_hemi(const float *p, const float *s, float *o, int n)
{
	for(int i = 0; i < n; ++i)
	{
		const float *q = p + 9 * i;
		const V3 r = cosHemisphere(v3(q[0], q[1], q[2]), v3(q[3], q[4], q[5]), v3(q[6], q[7], q[8]), s[2 * i], s[2 * i + 1]);
		o[3 * i] = r.x; o[3 * i + 1] = r.y; o[3 * i + 2] = r.z;
	}
}
void dm_coords(const float *in, float *o, int n)
{
	for(int i = 0; i < n; ++i)
	{
		V3 u, v;
		coordsSystem(v3(in[3 * i], in[3 * i + 1], in[3 * i + 2]), u, v);
		o[6 * i] = u.x; o[6 * i + 1] = u.y; o[6 * i + 2] = u.z; o[6 * i + 3] = v.x; o[6 * i + 4] = v.y; o[6 * i + 5] = v.z;
	}
}
void dm_normalize(const float *in, float *o, int n)
{
	for(int i = 0; i < n; ++i)
	{
		const V3 r = normalize(v3(in[3 * i], in[3 * i + 1], in[3 * i + 2]));
		o[3 * i] = r.x; o[3 * i + 1] = r.y; o[3 * i + 2] = r.z;
	}
}
void dm_mwc(uint32_t seed, int steps, double *o)
{
	Mwc m{30903u, seed};
	for(int i = 0; i < steps; ++i) o[i] = m.next();
}
// libm restatements (devmath.h libmAtan2f / libmAcosf) next to the host's own libm on the same inputs;
// the sphere mapping's long double expression next to real x87 long double
void dm_libm(const float *y, const float *x, int n, float *dev_atan2, float *libm_atan2, float *dev_acos, float *libm_acos)
{
	for(int i = 0; i < n; ++i)
	{
		dev_atan2[i] = libmAtan2f(y[i], x[i]);
		libm_atan2[i] = ::atan2f(y[i], x[i]);
		dev_acos[i] = libmAcosf(y[i]);
		libm_acos[i] = ::acosf(y[i]);
	}
}
void dm_sphere_v(const float *a, int n, float *dev, float *ref)
{
	const long double div_1_by_pi = 0.31830988618379067153776752674503L;   // include/math/math.h
	for(int i = 0; i < n; ++i)
	{
		dev[i] = x87oneMinus2Mul(kDiv1ByPi, a[i]);
		ref[i] = static_cast<float>(1.f - 2.f * (a[i] * div_1_by_pi));
	}
}
}
