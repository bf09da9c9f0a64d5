% krusell_smith_egm_gpu.m -- host script for the Krusell-Smith EGM solver (SURVEY §8(b) B6).
%
% Mirrors the ALM loop of Krusell_Smith_EGM.m:125-301 with its hot sections as gateway calls:
%   * the EGM policy iteration for the current ALM coefficients (:128-209) -> ks_egm_solve_mex
%       (Gauss-Seidel over (s, K) as the script: each column is overwritten as soon as it is
%        computed; pass jacobi = 1 as a 9th argument for the Jacobi variant, not the script's path)
%   * the shock panel (:57-93)                                              -> ks_shocks_mex (once)
%   * the panel simulation (:211-253)                                       -> ks_simulate_capital_mex
% The regressions of log K' on log K per aggregate state, the R^2 report and the damped update
% of B (:255-300) stay here.
% params = [beta alpha delta k_min k_max ug ub l_bar mu z_grid(1) z_grid(2) eps_grid(1) eps_grid(2)].

clear; clc;
% ---------------------------------------------------------------- parameters (:4-12)
beta = 0.99; alpha = 0.36; delta = 0.025; k_min = 0.0001; k_max = 1000;
k_size = 100; K_min = 30; K_max = 50; K_size = 4;
z_grid = [1.01, 0.99]; eps_grid = [1, 0];
ug = 0.04; ub = 0.10; mu = 0; l_bar = 1 / (1 - ub);
T = 1100; population = 10000; T_discard = 100;
max_iter_B = 100; tol_B = 1e-6; update_B = 0.3; max_egm = 10000; tol_egm = 1e-6;
params = [beta alpha delta k_min k_max ug ub l_bar mu z_grid eps_grid];

k_grid = linspace(0, 1, k_size).^7 * (k_max - k_min) + k_min;
k_grid(1) = k_min; k_grid(end) = k_max;
K_grid = linspace(K_min, K_max, K_size);

% ---------------------------------------------------------------- transition matrix (:22-54)
pgg = 1 - 1 / 8; pbb = 1 - 1 / 8; pgb = 1 - pgg; pbg = 1 - pbb;
p00_gg = 1 - 1 / 1.5; p00_bb = 1 - 1 / 2.5;
p00_gb = 1.25 * p00_bb; p00_bg = 0.75 * p00_gg;
p01_gg = 1 - p00_gg; p01_bb = 1 - p00_bb; p01_gb = 1 - p00_gb; p01_bg = 1 - p00_bg;
p10_gg = (ug - ug * p00_gg) / (1 - ug); p10_bb = (ub - ub * p00_bb) / (1 - ub);
p10_gb = (ub - ug * p00_gb) / (1 - ug); p10_bg = (ug - ub * p00_bg) / (1 - ub);
p11_gg = 1 - p10_gg; p11_bb = 1 - p10_bb; p11_gb = 1 - p10_gb; p11_bg = 1 - p10_bg;
P = [pgg * p11_gg, pgb * p11_gb, pgg * p10_gg, pgb * p10_gb;
     pbg * p11_bg, pbb * p11_bb, pbg * p10_bg, pbb * p10_bb;
     pgg * p01_gg, pgb * p01_gb, pgg * p00_gg, pgb * p00_gb;
     pbg * p01_bg, pbb * p01_bb, pbg * p00_bg, pbb * p00_bb];

% ---------------------------------------------------------------- shock panel (:56-93)
rng(5489, 'twister');
n_draws = (T - 1) + population + (T - 1) * population;
[zi_shock, epsi_shock] = ks_shocks_mex(T, population, rand(n_draws, 1), params);

% ---------------------------------------------------------------- ALM loop (:95-301)
k_opt = 0.9 * repmat(k_grid', [1, K_size, 4]);
B = [0, 1, 0, 1];
k_population = ones(population, 1) * K_grid(1);
for B_iter = 1:max_iter_B
    tic;
    [k_opt, egm_iter, egm_diff] = ks_egm_solve_mex(k_opt, k_grid, K_grid, B, P, params, ...
                                                   tol_egm, max_egm);
    [K_ts, k_population] = ks_simulate_capital_mex(k_opt, k_grid, K_grid, zi_shock, ...
                                                   epsi_shock, k_population);
    % OLS of log K(t+1) on [1, log K(t)] per aggregate state (t >= T_discard), with R^2
    t = (T_discard:T - 1)';
    good = zi_shock(t) == 0;
    B_new = zeros(1, 4); R2 = [0, 0];
    for g = [1, 0]
        sel = t(good == g);
        if ~isempty(sel)
            X = [ones(numel(sel), 1), log(K_ts(sel))];
            Y = log(K_ts(sel + 1));
            coef = X \ Y;
            B_new(3 - 2 * g:4 - 2 * g) = coef';
            resid = Y - X * coef;
            R2(2 - g) = 1 - sum(resid.^2) / sum((Y - mean(Y)).^2);
        end
    end
    diff_B = max(abs(B_new - B));
    fprintf(['ALM %3d: %d EGM sweeps (diff %.2e), B_new = [%.4f %.4f %.4f %.4f], diff %.2e, ' ...
             'R2 good %.4f bad %.4f (%.2f s)\n'], B_iter, egm_iter, egm_diff, B_new, diff_B, ...
            R2(1), R2(2), toc);
    if diff_B < tol_B
        break;
    end
    B = update_B * B_new + (1 - update_B) * B;
end
