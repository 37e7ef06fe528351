/*
 * tpch_gen.c -- deterministic synthetic TPC-H lineitem columns for the
 * oracle.  TEST INFRASTRUCTURE ONLY.
 *
 * The reference ships no dbgen and no lineitem.tbl for the
 * SF-0.01 known answers, so both the oracle and the product generate the
 * same counter-based columns: every value is a pure function of
 * (seed, row, column), so any row range can be produced independently
 * (shards, CPU samples) and the device generator in libmgdk.so must agree
 * with this one bit for bit (tested in tests/test_tpch_gen.py).
 *
 * Distributions follow the TPC-H specification (external spec, clause 4.2.3):
 *   o_orderdate  uniform in [1992-01-01, 1998-12-31 - 151 days]
 *   l_shipdate   = o_orderdate + U[1,121];  l_receiptdate = l_shipdate + U[1,30]
 *   l_quantity   U[1,50];  l_partkey U[1, SF*200000]
 *   p_retailprice = (90000 + ((pk/10) mod 20001) + 100*(pk mod 1000)) / 100
 *   l_extendedprice = l_quantity * p_retailprice
 *   l_discount   U[0.00,0.10];  l_tax U[0.00,0.08]
 *   l_returnflag 'R'/'A' (coin) if l_receiptdate <= 1995-06-17 else 'N'
 *   l_linestatus 'O' if l_shipdate > 1995-06-17 else 'F'
 * Decimals are stored as GDK lng with scale 2 (sql/common/sql_types.c:988-990),
 * dates as GDK packed dates (gdk/gdk_time.c:17-32), char(1) as 1-byte string
 * heap offsets (gdk/gdk_atoms.h:418-430): returnflag A=0,N=8,R=16;
 * linestatus F=0,O=8.
 */
#include "gdk_oracle.h"

static inline uint64_t
mix64(uint64_t z)
{
	/* splitmix64 finaliser */
	z += 0x9e3779b97f4a7c15ULL;
	z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
	z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
	return z ^ (z >> 31);
}

static inline uint64_t
rnd(uint64_t seed, uint64_t row, uint64_t col)
{
	return mix64(seed ^ mix64(row * 16 + col));
}

/* uniform integer in [lo, hi] via 64x64->128 multiply-high */
static inline int64_t
urange(uint64_t r, int64_t lo, int64_t hi)
{
	uint64_t span = (uint64_t) (hi - lo + 1);
	return lo + (int64_t) (((unsigned __int128) r * span) >> 64);
}

static const int cumdays[13] = {0, 31, 59, 90, 120, 151, 181, 212, 243, 273, 304, 334, 365};

static int
isleap(int y)
{
	return y % 4 == 0 && (y % 100 != 0 || y % 400 == 0);
}

int32_t
ora_mkdate(int y, int m, int d)
{
	/* gdk/gdk_time.c mkdate: ((y + 4712) * 12 + m - 1) << 5 | d */
	return (int32_t) ((((uint32_t) ((y + 4712) * 12 + m - 1)) << 5) | (uint32_t) d);
}

/* day number since 1992-01-01 -> packed date */
static int32_t
day2date(int day)
{
	int y = 1992;
	for (;;) {
		int len = 365 + isleap(y);
		if (day < len)
			break;
		day -= len;
		y++;
	}
	int m = 1;
	while (m < 12) {
		int end = cumdays[m] + (m >= 2 && isleap(y));
		if (day < end)
			break;
		m++;
	}
	int start = cumdays[m - 1] + (m > 2 && isleap(y));
	return ora_mkdate(y, m, day - start + 1);
}

#define ORDERDATE_DAYS 2405    /* 1998-08-02 - 1992-01-01 */
#define CURRENTDATE_DAY 1263   /* 1995-06-17 - 1992-01-01 */

void
ora_tpch_lineitem(uint64_t seed, uint64_t row0, uint64_t n, uint64_t sf_parts,
		  int32_t *shipdate, int64_t *quantity, int64_t *extendedprice,
		  int64_t *discount, int64_t *tax, uint8_t *returnflag,
		  uint8_t *linestatus)
{
	static int32_t table[ORDERDATE_DAYS + 121 + 30 + 2];
	static int init;
	if (!init) {
		for (int i = 0; i < (int) (sizeof(table) / sizeof(table[0])); i++)
			table[i] = day2date(i);
		init = 1;
	}
#pragma omp parallel for schedule(static)
	for (uint64_t i = 0; i < n; i++) {
		uint64_t row = row0 + i;
		int od = (int) urange(rnd(seed, row, 0), 0, ORDERDATE_DAYS);
		int sd = od + (int) urange(rnd(seed, row, 1), 1, 121);
		int rd = sd + (int) urange(rnd(seed, row, 2), 1, 30);
		int64_t q = urange(rnd(seed, row, 3), 1, 50);
		int64_t pk = urange(rnd(seed, row, 4), 1, (int64_t) sf_parts);
		int64_t rp = 90000 + ((pk / 10) % 20001) + 100 * (pk % 1000);
		if (shipdate)
			shipdate[i] = table[sd];
		if (quantity)
			quantity[i] = q * 100;
		if (extendedprice)
			extendedprice[i] = q * rp;
		if (discount)
			discount[i] = urange(rnd(seed, row, 5), 0, 10);
		if (tax)
			tax[i] = urange(rnd(seed, row, 6), 0, 8);
		if (returnflag)
			returnflag[i] = rd <= CURRENTDATE_DAY
				? ((rnd(seed, row, 7) >> 63) ? 16 /* R */ : 0 /* A */)
				: 8 /* N */;
		if (linestatus)
			linestatus[i] = sd > CURRENTDATE_DAY ? 8 /* O */ : 0 /* F */;
	}
}
