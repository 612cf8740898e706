"""Summarise rocprofv3 PMC results (rocpd sqlite) per kernel: counter -> mean value per dispatch."""
import collections, sqlite3, sys


def summary(path, match=""):
    c = sqlite3.connect(path)
    q = """select k.kernel_name, i.name, d.id, sum(p.value) from rocpd_pmc_event p
           join rocpd_info_pmc i on p.pmc_id = i.id
           join rocpd_kernel_dispatch d on d.event_id = p.event_id
           join rocpd_info_kernel_symbol k on d.kernel_id = k.id
           group by k.kernel_name, i.name, d.id"""
    acc = collections.defaultdict(list)
    for kn, name, _, v in c.execute(q):
        if match in kn:
            acc[(kn.split("(")[0], name)].append(v)
    return {k: sum(v) / len(v) for k, v in acc.items()}


if __name__ == "__main__":
    match = sys.argv[1]
    for p in sys.argv[2:]:
        for (kn, name), v in sorted(summary(p, match).items()):
            print(f"{kn[-40:]:40s} {name:26s} {v:16.1f}")
