"""Newton solver with step limiting: the MoorPy `dsolve2` RAFT's solveStatics calls
(raft/raft_model.py:771-772: tol = [0.05]*3 + [0.005]*3 per FOWT, a_max = 1.6,
maxIter = 20, RAFT's own step function).

MoorPy is third-party and absent here; this restates its published iteration:
  * evaluate Y(X); error = Y - Ytarget;
  * step dX = step_func(...) (RAFT: Newton on the total stiffness);
  * anti-oscillation: a step that re-crosses the plane at 0.62 of the previous step back
    is scaled to land on it;
  * convergence when every |dX_i| < tol_i -- the step is then NOT applied, so the returned
    X is the last evaluated point (its distance to the exact root is that last step);
  * at most maxIter evaluations.
"""
import numpy as np


def dsolve2(eval_func, X0, Ytarget=None, step_func=None, args=None, tol=1e-4, maxIter=20, a_max=2.0,
            Xmin=None, Xmax=None, display=0):
    X = np.array(np.atleast_1d(X0), dtype=float)
    N = len(X)
    Ytarget = np.zeros(N) if Ytarget is None or len(Ytarget) == 0 else np.asarray(Ytarget, dtype=float)
    tol = np.abs(np.broadcast_to(np.asarray(tol, dtype=float), (N,)))
    Xmin = np.full(N, -np.inf) if Xmin is None else np.asarray(Xmin, dtype=float)
    Xmax = np.full(N, np.inf) if Xmax is None else np.asarray(Xmax, dtype=float)
    Xs, Es = [], []
    dX_last = np.zeros(N)
    success = False
    Y = oths = None
    for it in range(maxIter):
        Y, oths, stop = eval_func(X, args)
        err = Y - Ytarget
        Xs.append(X.copy())
        Es.append(err.copy())
        if stop:
            break
        if it == maxIter - 1:
            if display > 0:
                print(f"dsolve2: no solution after {it} iterations, error {err}")
            break
        dX = np.asarray(step_func(X, args, Y, oths, Ytarget, err, tol, it, maxIter), dtype=float)
        # keep the iteration from reversing too much: do not re-cross the plane at
        # 0.62 of the previous step back
        Xlim = X - 0.62 * dX_last
        if np.sum((X + dX) * dX_last) < np.sum(Xlim * dX_last):
            alpha = np.sum((Xlim - X) * dX_last) / np.sum(dX * dX_last)
            dX = alpha * dX
        # bounds
        dX = np.where(X + dX < Xmin, Xmin - X, dX)
        dX = np.where(X + dX > Xmax, Xmax - X, dX)
        if np.all(np.abs(dX) < tol):
            success = True
            break
        dX_last = dX.copy()
        X = X + dX
    return X, Y, dict(iter=it, err=Y - Ytarget, dX=dX_last, oths=oths, Xs=np.array(Xs), Es=np.array(Es),
                      success=success)
