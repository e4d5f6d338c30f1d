/*
 * zoltan.h - source compatibility for programs written against the
 * reference dccrg, which call Zoltan_Initialize before creating a grid
 * (e.g. the reference's examples/game_of_life.cpp).  The MI355X framework
 * has no third-party partitioner (partitions are data: pins, export lists,
 * block partition), so initialization is all such a program needs.  Add
 * include/compat to the include path only when the real Zoltan is absent.
 */
#ifndef DCCRG_AMD_COMPAT_ZOLTAN_H
#define DCCRG_AMD_COMPAT_ZOLTAN_H

#define ZOLTAN_OK 0

static inline int Zoltan_Initialize(int argc, char** argv, float* version) {
	(void)argc;
	(void)argv;
	if (version) *version = 0.0f;
	return ZOLTAN_OK;
}

#endif
