"""Convert the reference's test instances into the committed LinProblem
fixtures under minotaur_amd/instances/ (run in the container that has
/root/reference; the GPU box only reads the .npz files).

  tls4_lin.npz     — linear rows of test_instances/tls4.nl
  tls4_oa.npz      — outer-approximation LP of tls4.nl: its four convex
                     -sum sqrt(x y) rows as tangent rows (config 2 as a MINLP;
                     minotaur_amd.problem.tls4_oa)
  knapsack9.npz    — OA-LP of examples/knapsack (config 3)
  color_lab2_qp.npz — QP relaxation data of test_instances/color_lab2_4x0.nl
                      (dense Q, equality rows; config 4)
  nvs08_oa.npz     — outer-approximation LP of test_instances/nvs08.nl
                      (config 1; minotaur_amd.problem.nvs08_oa)
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
from minotaur_amd.nl import read_nl            # noqa: E402
from minotaur_amd.problem import from_nl_linear, knapsack_oa, nvs08_oa, tls4_oa  # noqa: E402

REF = os.environ.get('MINOTAUR_REF', '/root/reference')
OUT = os.path.join(os.path.dirname(__file__), '..', 'minotaur_amd', 'instances')


def main():
    os.makedirs(OUT, exist_ok=True)
    tls4 = from_nl_linear(read_nl(os.path.join(REF, 'test_instances', 'tls4.nl')),
                          name='tls4-lin')
    tls4.save(os.path.join(OUT, 'tls4_lin.npz'))
    print('tls4-lin', tls4.n, tls4.m, tls4.nnz)
    oa = tls4_oa(read_nl(os.path.join(REF, 'test_instances', 'tls4.nl')))
    oa.save(os.path.join(OUT, 'tls4_oa.npz'))
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'oracle'))
    import oracle
    print('tls4-oa', oa.n, oa.m, oa.nnz, 'OA-MILP optimum (HiGHS)', oracle.highs_milp(oa))
    nv = nvs08_oa(read_nl(os.path.join(REF, 'test_instances', 'nvs08.nl')))
    nv.save(os.path.join(OUT, 'nvs08_oa.npz'))
    print('nvs08-oa', nv.n, nv.m, nv.nnz)
    ks = knapsack_oa()
    ks.save(os.path.join(OUT, 'knapsack9.npz'))
    print('knapsack9', ks.n, ks.m, ks.nnz)
    from minotaur_amd.qp import from_nl as qp_from_nl, save as qp_save
    cl = qp_from_nl(os.path.join(REF, 'test_instances', 'color_lab2_4x0.nl'),
                    name='color_lab2_4x0')
    qp_save(cl, os.path.join(OUT, 'color_lab2_qp.npz'))
    print('color_lab2 QP', cl.n, cl.m)


if __name__ == '__main__':
    main()
