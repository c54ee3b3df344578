// Development profile builds of the sort kernel (tools/build_variant.py NAME
// -DSVS_FOLD_PROF or -DSVS_FOLD_PROF_EXAM; SVS_POA_FOLD_TIMES=1 prints the
// totals).  The product build compiles every macro below to nothing.
//   SVS_FOLD_PROF:      prof[0] fast-root clocks, prof[1] DFS-run clocks,
//                       prof[2] / prof[3] new- / old-node window loads
//   SVS_FOLD_PROF_EXAM: prof[0..3] the DFS examination's phases (record, flag
//                       reads, pushes/emits, pop), in clocks
// (used inside dfs_sort, where S is the SortState)
#pragma once

#if defined(SVS_FOLD_PROF) || defined(SVS_FOLD_PROF_EXAM)
#define SVS_PF_CLK() __builtin_readcyclecounter()
#else
#define SVS_PF_CLK() 0ull
#endif
#ifdef SVS_FOLD_PROF_EXAM
#define SVS_PF_COUNT(k) ((void)0)
#define SVS_PF_ADD(k, t) ((void)0)
#define SVS_PF_EXAM(k, t) (S.prof[k] += SVS_PF_CLK() - (t))
#define SVS_PF_SHIFT(k) 10
#else
#define SVS_PF_COUNT(k) (S.prof[k] += 1)
#define SVS_PF_ADD(k, t) (S.prof[k] += SVS_PF_CLK() - (t))
#define SVS_PF_EXAM(k, t) ((void)0)
#define SVS_PF_SHIFT(k) ((k) < 2 ? 10 : 0)
#endif
